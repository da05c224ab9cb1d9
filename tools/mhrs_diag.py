#!/usr/bin/env python3
"""MHRS attempt-search lane utilisation from a -D PHT_MHRS_DIAG variant build
(PHT_LIB): lane iterations with an attempt / (64 x wavefront iterations),
overall and for rounds 0 and 1, and the share of wavefront iterations with
at most 8 lanes working (a round's tail).  One sweep at the generating
parameters (close to the posterior, i.e. past burn-in).
usage (GPU box): PHT_LIB=phasetype_amd/_variants/mdiag.so python3 tools/mhrs_diag.py [--n 10 --N 1000000 --censor 0]"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import phasetype_amd as P  # noqa: E402
from phasetype_amd.synth import DATA_KEY, bd_exit, simulate_ph  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--n", type=int, default=10)
ap.add_argument("--N", type=int, default=1_000_000)
ap.add_argument("--censor", type=float, default=0.0)
a = ap.parse_args()
S, s = bd_exit(a.n)
y, cen = simulate_ph(S, s, a.N, seed=DATA_KEY, censor_frac=a.censor)
sw = P.Sweeper(a.n, 1)
sw.set_obs(y, cen)
for k in range(3):
    st = sw.sweep(S, s, key=(1, 2), sweep=1 + k, zexp=P.zexp_for(y))
    _, _, _, ex = P.split_stats(st, a.n)
    w, l, t = float(ex[8]), float(ex[9]), float(ex[10])
    print(json.dumps({"n": a.n, "N": a.N, "censor": a.censor, "sweep": 1 + k, "kernel_ms": sw.last_kernel_ms(),
                      "attempts": int(ex[1]), "lane_util_search": l / max(1.0, 64 * w),
                      "tail_wave_iter_frac": t / max(1.0, w),
                      "lane_util_round0": float(ex[12]) / max(1.0, 64 * float(ex[11])),
                      "lane_util_round1": float(ex[14]) / max(1.0, 64 * float(ex[13])),
                      "wave_iters": int(w), "wave_iters_round0": int(ex[11]), "wave_iters_round1": int(ex[13])}))
