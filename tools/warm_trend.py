#!/usr/bin/env python3
"""Kernel time per sweep against wall time at FIXED parameters: does the same
work get faster as the process keeps the GPU busy (clock / power ramp, or
anything else time-dependent)?  Fixed (S, s) = BD-exit(n) truth, the same
observations, sweep index varied (different draws, same law).

usage (GPU box): python3 tools/warm_trend.py [--method ECS] [--n 10] [--N 1000000] [--sweeps 600]
Prints one JSON line per bucket of 20 sweeps (mean kernel ms, wall ms per
sweep, elapsed s) and a summary.
"""
import argparse
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import phasetype_amd as P  # noqa: E402
from phasetype_amd.synth import DATA_KEY, bd_exit, simulate_ph  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--method", default="ECS")
    ap.add_argument("--n", type=int, default=10)
    ap.add_argument("--N", type=int, default=1_000_000)
    ap.add_argument("--censor", type=float, default=0.0)
    ap.add_argument("--sweeps", type=int, default=600)
    ap.add_argument("--bucket", type=int, default=20)
    a = ap.parse_args()
    S, s = bd_exit(a.n)
    y, cen = simulate_ph(S, s, a.N, seed=DATA_KEY, censor_frac=a.censor)
    zexp = P.zexp_for(y)
    sw = P.Sweeper(a.n, P.METHODS[a.method], 1)
    sw.set_obs(y, cen)
    t00 = time.perf_counter()
    ks, ws = [], []
    for it in range(a.sweeps):
        t0 = time.perf_counter()
        sw.sweep(S, s, key=(3, 5), sweep=it + 1, zexp=zexp)
        ws.append((time.perf_counter() - t0) * 1e3)
        ks.append(sw.last_kernel_ms())
        if (it + 1) % a.bucket == 0:
            print(json.dumps({"sweeps": it + 1, "elapsed_s": round(time.perf_counter() - t00, 3),
                              "kernel_ms": round(float(np.mean(ks[-a.bucket:])), 4),
                              "wall_ms": round(float(np.mean(ws[-a.bucket:])), 4)}), flush=True)
    print(json.dumps({"method": a.method, "n": a.n, "N": a.N, "first_bucket_kernel_ms": float(np.mean(ks[:a.bucket])),
                      "last_bucket_kernel_ms": float(np.mean(ks[-a.bucket:])),
                      "min_kernel_ms": float(np.min(ks))}), flush=True)
    sw.close()


if __name__ == "__main__":
    main()
