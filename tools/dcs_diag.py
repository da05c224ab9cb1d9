#!/usr/bin/env python3
"""Lane utilisation of the DCS kernel's loops from a PHT_DCS_DIAG build
(tools/build_variant.py diag -D PHT_DCS_DIAG; run with PHT_LIB=<that .so>):
lane Brent evaluations / (64 x wavefront Brent iterations), lane jumps /
(64 x wavefront rounds).  usage (GPU box): python3 tools/dcs_diag.py [--n 10]"""
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
ap.add_argument("--N", type=int, default=500000)
a = ap.parse_args()
S, s = bd_exit(a.n)
y, cen = simulate_ph(S, s, a.N, seed=DATA_KEY, censor_frac=0.3)
sw = P.Sweeper(a.n, 4)
sw.set_obs(y, cen)
zexp = P.zexp_for(y)
st = sw.sweep(S, s, key=(3, 4), zexp=zexp)
ex = st[2 * a.n + a.n * a.n:]
print(json.dumps({"n": a.n, "N": a.N, "kernel_ms": sw.last_kernel_ms(), "obs": int(ex[0]), "jumps": int(ex[4]),
                  "brent_evals": int(ex[5]), "wave_brent_iters": int(ex[6]), "wave_rounds": int(ex[7]),
                  "brent_lane_util": float(ex[5]) / max(1.0, 64.0 * float(ex[6])),
                  "round_lane_util": float(ex[4]) / max(1.0, 64.0 * float(ex[7]))}))
