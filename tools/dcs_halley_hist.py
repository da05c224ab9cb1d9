#!/usr/bin/env python3
"""Evaluations per DCS jump of the device spec's Halley root (the oracle's dev
variant, bit-identical to pht_dcs_round.h hob_halley), and the expected
maximum over a wavefront's 64 lanes — what a jump-converged round waits for.
Diagnostic (CPU only).

usage: python3 tools/dcs_halley_hist.py [--N 20000] > profiles/.../halley.json
"""
import argparse
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from oracle.oracle import OracleLib  # noqa: E402
from phasetype_amd.synth import DATA_KEY, bd_exit, simulate_ph  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--N", type=int, default=20000)
    a = ap.parse_args()
    o = OracleLib()
    out = []
    for n, cf in ((5, 0.3), (10, 0.0), (15, 0.3), (20, 0.0)):
        S, s = bd_exit(n)
        y, cen = simulate_ph(S, s, a.N, seed=DATA_KEY, censor_frac=cf)
        o.halley_hist()
        o.dev_sweep(4, S, s, y, cen, per_obs=False)
        h = o.halley_hist().astype(float)
        p = h / h.sum()
        cdf = np.cumsum(p)
        out.append({"n": n, "N": a.N, "censor": cf, "jumps": int(h.sum()),
                    "mean_evals": float((np.arange(64) * p).sum()),
                    "expected_max_of_64": float(sum(1 - cdf[k] ** 64 for k in range(64))),
                    "frac_ge6": float(p[6:].sum()),
                    "hist": {int(k): int(v) for k, v in enumerate(h) if v}})
        print(json.dumps(out[-1]), flush=True)


if __name__ == "__main__":
    main()
