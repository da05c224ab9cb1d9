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


class _FakeSweeper:
    """Stands in for a GPU Sweeper in attach_rccl's failure paths (no GPU
    here): attach fails on the ranks listed, the library all-reduce is
    never reached."""

    def __init__(self, fail_attach, fail_prepare=False):
        self.fail_attach = fail_attach
        self.fail_prepare = fail_prepare
        self.attach_called = False

    def rccl_prepare(self, max_len):
        if self.fail_prepare:
            raise RuntimeError("librccl.so.1 could not be loaded (fake)")

    def attach_rccl(self, uid, world, rank):
        self.attach_called = True
        if self.fail_attach:
            raise RuntimeError("ncclCommInitRank failed (fake)")

    def rccl_allreduce(self, buf):
        raise RuntimeError("not attached (fake)")


def _attach_worker(rank, world, port, mode):
    import sys

    sys.path.insert(0, REPO)
    import torch.distributed as dist

    import phasetype_amd as P
    from phasetype_amd import dist as D

    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    try:
        if mode == "no_id":  # rank 0 cannot make an RCCL id
            def boom():
                raise RuntimeError("no RCCL (fake)")
            P.rccl_unique_id = boom
            sw = _FakeSweeper(False)
        elif mode == "prepare_fails_on_one_rank":  # a local precondition fails on the last rank
            P.rccl_unique_id = lambda: bytes(P.RCCL_ID_BYTES)
            sw = _FakeSweeper(False, fail_prepare=rank == world - 1)
        else:  # the communicator fails on the last rank only
            P.rccl_unique_id = lambda: bytes(P.RCCL_ID_BYTES)
            sw = _FakeSweeper(rank == world - 1)
        assert D.attach_rccl(sw, dist, "cpu") is False
        if mode == "prepare_fails_on_one_rank":
            # nobody may enter the collective ncclCommInitRank
            assert not sw.attach_called
        dist.barrier()
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("mode", ["no_id", "prepare_fails_on_one_rank", "attach_fails_on_one_rank"])
def test_attach_rccl_failures_fall_back_on_every_rank(mode):
    """bench.py's in-library RCCL reduce: a failure on any rank (no RCCL id
    on rank 0, a communicator that fails on one rank) must return False on
    every rank — the callback reduce is then used — instead of leaving the
    other ranks waiting in a collective."""
    import torch.multiprocessing as mp

    mp.spawn(_attach_worker, args=(2, _free_port(), mode), nprocs=2, join=True)
