#!/usr/bin/env python3
"""Debug helper (GPU box): per-observation GPU vs oracle for one small ECS
case with PHT_ROWK forced; prints the differing observations' fields.
usage: python3 tools/dbg_rows.py N n rowk [censor] [yscale] [seed]"""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import phasetype_amd as P  # noqa: E402
from oracle import oracle as O  # noqa: E402
from phasetype_amd.synth import bd_exit, simulate_ph  # noqa: E402

N, n, rowk = int(sys.argv[1]), int(sys.argv[2]), sys.argv[3]
cf = float(sys.argv[4]) if len(sys.argv) > 4 else 0.3
ysc = float(sys.argv[5]) if len(sys.argv) > 5 else 1.0
seed = int(sys.argv[6]) if len(sys.argv) > 6 else 900 + N
os.environ["PHT_ROWK"] = rowk
orc = O.OracleLib()
S, s = bd_exit(n)
y, cen = simulate_ph(S, s, N, seed=seed, censor_frac=cf)
y = y * ysc
y = np.ascontiguousarray(y, np.float64)
cen = np.ascontiguousarray(cen, np.int32)
zexp = int(orc.lib.orc_zexp(y, len(y)))
sw = P.Sweeper(n, 2, 1)
sw.set_obs(y, cen)
t0 = time.time()
g = sw.sweep_debug(S, s, key=(3, 5), sweep=2, zexp=zexp)
t1 = time.time()
o = orc.dev_sweep(2, S, s, y, cen, key=(3, 5), sweep=2, zexp=zexp)
print("gpu s", round(t1 - t0, 3))
bad = sorted(set(np.nonzero((g["pre"] != o["pre"]) | (g["ndraw"] != o["ndraw"]) | (g["B"] != o["B"]))[0]))
print("bad", len(bad), "of", N, "exact", int((cen == 0).sum()))
for i in bad[:8]:
    print(i, "y", y[i], "cen", cen[i], "pre", g["pre"][i], o["pre"][i], "ndraw", g["ndraw"][i], o["ndraw"][i],
          "flags", g["flags"][i], o["flags"][i], "zq", g["zq"][i], o["zq"][i])
