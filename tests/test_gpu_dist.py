"""GPU: bench.py's RCCL path, run under torchrun with one rank.

The driver's scaling runs launch bench.py under torchrun with N > 1 ranks;
the multi-rank arithmetic of phasetype_amd/dist.py is covered over gloo in
test_multirank.py.  Here torchrun starts ONE rank on the GPU, which (WORLD_SIZE
set) initialises the "nccl" (RCCL) process group and, with
PHT_WORLD1_REDUCE=1, goes through the same code as N > 1: the statistics all-reduce every sweep (RCCL on the sweep
stream inside the library, Sweeper.attach_rccl), max-over-ranks timing, the
weak-scaling side measurement.  It runs in a child process because
torch must initialise the device before the library loads (bench.py's order;
this pytest process loaded the library first).
"""
import json
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.parametrize("reduce_at_world1", [True, False])
def test_bench_under_torchrun_rccl(gpu, reduce_at_world1):
    """With PHT_WORLD1_REDUCE=1 the one rank runs the N > 1 statistics path
    (RCCL all-reduce on the sweep stream, self-tested at attach); by default
    a world of one runs no collective (bench.py use_coll)."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "1",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
           os.path.join(REPO, "bench.py"), "--gpus", "1", "--steps", "4", "--warmup", "1",
           "--N", "200000", "--no-cpu-baseline"]
    env = dict(os.environ, PHT_WORLD1_REDUCE="1" if reduce_at_world1 else "0")
    p = subprocess.run(cmd, cwd=REPO, capture_output=True, text=True, timeout=240, env=env)
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, p.stdout[-2000:]
    line = json.loads(lines[0])
    assert line["n_gpus"] == 1 and line["steps"] == 4
    assert line["value"] > 0 and line["ms_per_step"] > 0
    assert line["weak_scaling"]["N_total"] == 200000
    want = "rccl-in-stream (self-tested)" if reduce_at_world1 else "none (world 1)"
    assert line["config"]["stats_reduce"] == want


def _chain_child(nproc):
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(nproc),
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
           os.path.join(REPO, "tests", "_rccl_chain_child.py")]
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    p = subprocess.run(cmd, cwd=REPO, capture_output=True, text=True, timeout=240, env=env)
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, p.stdout[-2000:]
    got = json.loads(lines[0])
    want = {f"{k}_{v}": True for k in ("ECS_n5", "MHRS_n4", "DCS_n4") for v in ("rccl", "callback")}
    want["selftest"] = True
    assert got == want, got


def test_rccl_in_stream_reduce_keeps_the_chain(gpu):
    """Sweeper.attach_rccl (pht_ctx_attach_rccl) with one rank: its
    self-test passes, and the chain with the statistics summed by RCCL on the
    sweep stream (and with the host callback) equals the chain without any
    reduce."""
    _chain_child(1)


def test_rccl_two_ranks_equal_single_shard(gpu):
    """Two ranks on two GPUs: the in-library RCCL sum and the host-callback
    sum both give the single-process chain over all observations, draw for
    draw (the N > 1 default path).  Needs two visible GPUs."""
    if gpu < 2:
        pytest.skip("needs 2 GPUs (the driver's 8-GPU node; the 1-GPU box cannot host two RCCL ranks)")
    _chain_child(2)
