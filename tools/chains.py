#!/usr/bin/env python3
"""Throughput of independent chains at once (pht_gibbs_run_chains,
SURVEY.md §8f.4) against one chain, at the small configurations where one
chain leaves the GPU mostly idle.  Time per sweep from the difference of two
runs (it = 101 and 21), so context setup and uploads cancel.
usage (GPU box): python3 tools/chains.py [--Ks 1 2 4 8]"""
import argparse
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import phasetype_amd as P  # noqa: E402
from phasetype_amd.synth import DATA_KEY, bd_exit, bd_exit_structure, simulate_ph  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--Ks", nargs="+", type=int, default=[1, 2, 4, 8])
    ap.add_argument("--cfgs", nargs="+", default=["cfg1:3:200:ECS", "cfg2:5:10000:ECS", "cfg2m:5:10000:MHRS", "cfg2d:5:10000:DCS", "cfg2u:5:10000:UNIF"])
    a = ap.parse_args()
    for spec in a.cfgs:
        name, n, N, meth = spec.split(":")
        n, N, method = int(n), int(N), P.METHODS[meth]
        S, s = bd_exit(n)
        T, theta = bd_exit_structure(n)
        nu, zeta = 1 + 50 * theta, np.full(len(theta), 50.0)
        y, cen = simulate_ph(S, s, N, seed=DATA_KEY)
        out = {"config": name, "n": n, "N": N, "method": meth}
        P.gibbs_chains([1], y, cen, n, method, nu, zeta, T, np.ones(T.shape), it=5)  # warm-up
        for K in a.Ks:
            seeds = list(range(1, K + 1))
            best = []
            for rep in range(3):
                ts = []
                for it in (21, 101):
                    t0 = time.perf_counter()
                    P.gibbs_chains(seeds, y, cen, n, method, nu, zeta, T, np.ones(T.shape), it=it)
                    ts.append(time.perf_counter() - t0)
                best.append((ts[1] - ts[0]) / 80)
            per_sweep = float(np.median(best))
            out[f"K{K}"] = {"ms_per_sweep": round(per_sweep * 1e3, 4),
                            "chain_sweeps_per_s": round(K / per_sweep, 1)}
        print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
