"""Child of test_gpu_dist.py (run under torchrun, 1 or more ranks, RCCL,
one GPU per rank): each rank sweeps its shard; the chain with the statistics
block summed by the in-library RCCL all-reduce (Sweeper.attach_rccl, after
its self-test) and the chain with the host callback (make_stats_allreduce)
both equal the single-process chain over ALL observations (computed on every
rank without any reduce), draw for draw.  Prints one JSON line on rank 0."""
import json
import os
import sys

import numpy as np
import torch
import torch.distributed as dist

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

local = int(os.environ.get("LOCAL_RANK", "0"))
torch.cuda.set_device(local)
dist.init_process_group("nccl", device_id=torch.device("cuda", local))

import phasetype_amd as P  # noqa: E402
from phasetype_amd.dist import attach_rccl, make_stats_allreduce, shard_range  # noqa: E402
from phasetype_amd.synth import bd_exit, bd_exit_structure, simulate_ph  # noqa: E402

dev = f"cuda:{local}"
out = {"selftest": True}
for n, method, cf in ((5, "ECS", 0.3), (4, "MHRS", 0.0), (4, "DCS", 0.0)):
    S, s = bd_exit(n)
    T, theta = bd_exit_structure(n)
    m = len(theta)
    nu, zeta = 1.0 + 50.0 * theta, np.full(m, 50.0)
    y, cen = simulate_ph(S, s, 20000, seed=77 + n, censor_frac=cf)
    zexp = P.zexp_for(y)
    lo, hi = shard_range(len(y), dist.get_rank(), dist.get_world_size())
    meth = P.METHODS[method]

    def run(mode):
        if mode == "single":
            sw = P.Sweeper(n, meth, 1, device=local)
            sw.set_obs(y, cen)
        else:
            sw = P.Sweeper(n, meth, 1, device=local)
            sw.set_obs(y[lo:hi], cen[lo:hi], obs0=lo)
            sw.set_global_count(len(y))
        red = None
        if mode == "rccl":
            out["selftest"] &= attach_rccl(sw, dist, dev)
            try:  # a callback on top of the attached communicator would sum twice: refused
                sw.gibbs(2, meth, nu, zeta, T, np.ones(T.shape), zexp, reduce=lambda a: None)
                out["selftest"] = False
            except P.PhaseTypeError as e:
                out["selftest"] &= "RCCL communicator attached" in str(e)
        elif mode == "callback":
            red = make_stats_allreduce(dist, P.stats_len(n), device=dev)
        P.set_seed(4242)
        r = sw.gibbs(6, meth, nu, zeta, T, np.ones(T.shape), zexp, reduce=red)
        sw.close()
        return r

    want = run("single")
    for mode in ("rccl", "callback"):
        got = run(mode)
        out[f"{method}_n{n}_{mode}"] = bool(np.array_equal(want, got)) and bool(np.all(np.isfinite(got)))
dist.barrier()
dist.destroy_process_group()
if int(os.environ.get("RANK", "0")) == 0:
    print(json.dumps(out))
