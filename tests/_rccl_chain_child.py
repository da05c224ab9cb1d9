"""Child of test_gpu_dist.py (run under torchrun, one rank, RCCL): the chain
with the statistics block summed by the in-library RCCL all-reduce
(Sweeper.attach_rccl) equals the chain without any reduce, draw for draw.
Prints one JSON line."""
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
from phasetype_amd.dist import attach_rccl, shard_range  # noqa: E402
from phasetype_amd.synth import bd_exit, bd_exit_structure, simulate_ph  # noqa: E402

out = {}
for n, method, cf in ((5, "ECS", 0.3), (4, "MHRS", 0.0), (4, "DCS", 0.0)):
    S, s = bd_exit(n)
    T, theta = bd_exit_structure(n)
    m = len(theta)
    nu, zeta = 1.0 + 50.0 * theta, np.full(m, 50.0)
    y, cen = simulate_ph(S, s, 20000, seed=77 + n, censor_frac=cf)
    zexp = P.zexp_for(y)
    lo, hi = shard_range(len(y), dist.get_rank(), dist.get_world_size())
    res = []
    for attach in (False, True):
        sw = P.Sweeper(n, P.METHODS[method], 1, device=local)
        sw.set_obs(y[lo:hi], cen[lo:hi], obs0=lo)
        if attach:
            attach_rccl(sw, dist, f"cuda:{local}")
        P.set_seed(4242)
        res.append(sw.gibbs(6, P.METHODS[method], nu, zeta, T, np.ones(T.shape), zexp))
        sw.close()
    out[f"{method}_n{n}"] = bool(np.array_equal(res[0], res[1])) and bool(np.all(np.isfinite(res[1])))
dist.barrier()
dist.destroy_process_group()
print(json.dumps(out))
