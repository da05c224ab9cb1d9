"""CPU, world_size 2, 3 and 8 (the driver's largest node) over gloo: the
multi-process sharding of phasetype_amd/dist.py (the code bench.py runs over RCCL on the GPUs).

Each rank sweeps its shard_range() of the observations with the device
specification (oracle "dev" variant, global observation ids = obs0 offsets,
exactly what a GPU shard computes) and the int64 statistics blocks are summed
with make_stats_allreduce().  Bar: every rank ends with the block of a single
sweep over all observations, bit for bit — so the Gibbs chain (drawn from the
summed block with the same host stream on every rank) is identical for every
world size.
"""
import os
import socket

import numpy as np
import pytest

from phasetype_amd.dist import shard_range
from phasetype_amd.synth import bd_exit, simulate_ph

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _block(o, n):
    """oracle dev_sweep totals -> the kernels' int64 stats layout."""
    st = np.zeros(2 * n + n * n + 16, np.int64)
    st[:n] = o["zq_tot"]
    st[n:2 * n] = o["B_tot"]
    st[2 * n:2 * n + n * n] = o["N_tot"].T.reshape(-1)  # N[i + j n]
    return st


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, cases):
    import sys

    sys.path.insert(0, REPO)
    import torch.distributed as dist

    from oracle.oracle import OracleLib
    from phasetype_amd.dist import make_stats_allreduce, max_over_ranks, sum_over_ranks

    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    try:
        orc = OracleLib()
        for n, N, method, cf in cases:
            S, s = bd_exit(n)
            y, cen = simulate_ph(S, s, N, seed=123 + n, censor_frac=cf)
            zexp = int(orc.lib.orc_zexp(np.ascontiguousarray(y), len(y)))
            reduce = make_stats_allreduce(dist, 2 * n + n * n + 16)
            for sweep in (1, 2):
                lo, hi = shard_range(N, rank, world)
                part = orc.dev_sweep(method, S, s, y[lo:hi], cen[lo:hi], key=(9, 10), sweep=sweep, zexp=zexp,
                                     obs0=lo, per_obs=False)
                st = _block(part, n)
                reduce(st)
                full = orc.dev_sweep(method, S, s, y, cen, key=(9, 10), sweep=sweep, zexp=zexp, per_obs=False)
                want = _block(full, n)
                assert np.array_equal(st, want), (rank, n, method, sweep)
        mx = max_over_ranks(dist, [float(rank), -float(rank)])
        assert mx == [float(world - 1), 0.0]
        sm = sum_over_ranks(dist, [float(rank + 1)])
        assert sm == [world * (world + 1) / 2.0]
        dist.barrier()
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3, 8])
def test_sharded_sweeps_sum_to_single_sweep(orc, world):
    import torch.multiprocessing as mp

    cases = [(4, 3001, 2, 0.3), (4, 2000, 1, 0.3), (3, 1500, 4, 0.0)]
    mp.spawn(_worker, args=(world, _free_port(), cases), nprocs=world, join=True)


def test_shard_range_partitions():
    for N in (0, 1, 7, 1000003):
        for world in (1, 2, 3, 8):
            r = [shard_range(N, k, world) for k in range(world)]
            assert r[0][0] == 0 and r[-1][1] == N
            assert all(a[1] == b[0] for a, b in zip(r, r[1:]))
            assert max(h - lo for lo, h in r) - min(h - lo for lo, h in r) <= 1
