#!/usr/bin/env python3
"""ECS round diagnostics from a -D PHT_ECS_DIAG variant build (PHT_LIB):
how often lanes run the general ARMS code (envelope beyond the converged
round's 13 points) and how many wave-rounds that divergence touches, and
the width the converged blocks run at (9, 11 or 13 points: the widest
envelope in the wavefront; word 5 counts the 13-point wave-rounds).
usage (GPU box): PHT_LIB=phasetype_amd/_variants/diag.so python3 tools/ecs_diag.py [--n 10 --N 1000000]"""
import argparse
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import phasetype_amd as P  # noqa: E402
from phasetype_amd.synth import DATA_KEY, bd_exit, simulate_ph  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--n", type=int, default=10)
ap.add_argument("--N", type=int, default=1_000_000)
ap.add_argument("--rowk", type=int, default=0, help="PHT_ROWK (the diag counters cover the one-lane blocks)")
a = ap.parse_args()
os.environ["PHT_ROWK"] = str(a.rowk)
S, s = bd_exit(a.n)
y, cen = simulate_ph(S, s, a.N, seed=DATA_KEY)
sw = P.Sweeper(a.n, 2)
sw.set_obs(y, cen)
st = sw.sweep(S, s, key=(1, 2), sweep=1, zexp=P.zexp_for(y))
_, _, _, ex = P.split_stats(st, a.n)
print(json.dumps({"n": a.n, "N": a.N, "kernel_ms": sw.last_kernel_ms(), "obs": int(ex[0]), "jumps": int(ex[4]),
                  "lane_rounds_big": int(ex[6]), "wave_rounds_with_big": int(ex[7]), "wave_rounds": int(ex[8]),
                  "lane_rounds_active": int(ex[9]), "lane_rounds_start": int(ex[10]),
                  "lane_rounds_pend": int(ex[11]), "lane_rounds_newobs": int(ex[12]),
                  "wave_rounds_with_newobs": int(ex[13]), "wave_rounds_with_pend": int(ex[14]),
                  "wave_rounds_cap13": int(ex[5]),
                  "frac_wave_rounds_cap13": float(ex[5]) / max(1.0, float(ex[8])),
                  "frac_wave_rounds_cap11": float(ex[14] - ex[5]) / max(1.0, float(ex[8])),
                  "active_lane_frac": float(ex[9]) / max(1.0, 64.0 * float(ex[8])),
                  "frac_wave_rounds_with_big": float(ex[7]) / max(1.0, float(ex[8])),
                  "big_per_jump": float(ex[6]) / max(1.0, float(ex[4]))}))
