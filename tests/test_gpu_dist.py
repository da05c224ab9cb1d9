"""GPU: bench.py's RCCL path, run under torchrun with one rank.

The driver's scaling runs launch bench.py under torchrun with N > 1 ranks;
the multi-rank arithmetic of phasetype_amd/dist.py is covered over gloo in
test_multirank.py.  Here torchrun starts ONE rank on the GPU, which (WORLD_SIZE
set) initialises the "nccl" (RCCL) process group and goes through the same
code as N > 1: the statistics all-reduce every sweep (RCCL on the sweep
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


def test_bench_under_torchrun_rccl(gpu):
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "1",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
           os.path.join(REPO, "bench.py"), "--gpus", "1", "--steps", "4", "--warmup", "1",
           "--N", "200000", "--no-cpu-baseline"]
    p = subprocess.run(cmd, cwd=REPO, capture_output=True, text=True, timeout=240)
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, p.stdout[-2000:]
    line = json.loads(lines[0])
    assert line["n_gpus"] == 1 and line["steps"] == 4
    assert line["value"] > 0 and line["ms_per_step"] > 0
    assert line["weak_scaling"]["N_total"] == 200000
    assert line["config"]["stats_reduce"] == "rccl-in-stream"


def test_rccl_in_stream_reduce_keeps_the_chain(gpu):
    """Sweeper.attach_rccl (pht_ctx_attach_rccl): the statistics block summed
    by RCCL on the sweep stream gives the same chain as no reduce (one rank)."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "1",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
           os.path.join(REPO, "tests", "_rccl_chain_child.py")]
    p = subprocess.run(cmd, cwd=REPO, capture_output=True, text=True, timeout=240)
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, p.stdout[-2000:]
    got = json.loads(lines[0])
    assert got == {"ECS_n5": True, "MHRS_n4": True, "DCS_n4": True}, got
