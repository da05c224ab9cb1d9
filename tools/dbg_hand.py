#!/usr/bin/env python3
"""Diagnostic (GPU box): the ECS hand-off against the oracle, per field.
usage: python3 tools/dbg_hand.py [n] [N] [hand]"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import phasetype_amd as P  # noqa: E402
from oracle import oracle as O  # noqa: E402
from phasetype_amd.synth import bd_exit, simulate_ph  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 10
N = int(sys.argv[2]) if len(sys.argv) > 2 else 20000
hand = sys.argv[3] if len(sys.argv) > 3 else "3"
orc = O.OracleLib()
S, s = bd_exit(n)
y, cen = simulate_ph(S, s, N, seed=7000 + n)
zexp = P.zexp_for(y)
o = orc.dev_sweep(2, S, s, y, cen, key=(5, 6), sweep=3, zexp=zexp)
for h in ("0", hand):
    os.environ["PHT_HAND"] = h
    os.environ["PHT_HANDBLK"] = "8"
    sw = P.Sweeper(n, 2, 1)
    sw.set_obs(y, cen)
    g = sw.sweep_debug(S, s, key=(5, 6), sweep=3, zexp=zexp)
    sw.close()
    bad = {f: np.nonzero(g[f] != o[f])[0] for f in ("B", "pre", "flags", "ndraw")}
    bz = np.nonzero(np.any(g["zq"] != o["zq"], axis=1))[0]
    bN = np.nonzero(np.any(g["N"].reshape(N, -1) != o["N"].reshape(N, -1), axis=1))[0]
    print("hand", h, {f: len(v) for f, v in bad.items()}, "z", len(bz), "N", len(bN), "obs", P.split_stats(g["stats"], n)[3][0])
    if len(bad["pre"]):
        i = bad["pre"][:6]
        print("  pre gpu", g["pre"][i], "orc", o["pre"][i], "ndraw gpu", g["ndraw"][i], "orc", o["ndraw"][i])
        print("  jumps gpu", (g["N"][i].sum(axis=(1, 2)) - np.trace(g["N"][i], axis1=1, axis2=2)),
              "orc", (o["N"][i].sum(axis=(1, 2)) - np.trace(o["N"][i], axis1=1, axis2=2)))
        print("  z sum gpu", g["zq"][i].sum(1) * 2.0 ** -zexp, "orc", o["zq"][i].sum(1) * 2.0 ** -zexp, "y", y[i])
