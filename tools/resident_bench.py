#!/usr/bin/env python3
"""Sweeps/s of the device-resident chain (pht_gibbs_run_resident) next to
the host-loop chain (pht_gibbs_run) with the same sampler (ECS, DCS at cfg5,
UNIF, MHRS), at BASELINE.json's single-GPU configurations; argv: config
names and/or methods to restrict to.
Prints one JSON line per (config, mode).  Run on the GPU box."""
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import phasetype_amd as P  # noqa: E402
from phasetype_amd.synth import DATA_KEY, bd_exit, bd_exit_structure, simulate_ph  # noqa: E402

CFGS = [("cfg1", 3, 200, 0.0, 2000), ("cfg2", 5, 10_000, 0.0, 1000), ("cfg3", 20, 100_000, 0.0, 200),
        ("cfg4", 10, 1_000_000, 0.0, 100), ("cfg5", 15, 500_000, 0.3, 100)]
want = set(sys.argv[1:])
for name, n, N, cf, steps in CFGS:
    if want - set(P.METHODS) and name not in want:
        continue
    S, s = bd_exit(n)
    T, theta = bd_exit_structure(n)
    nu, zeta, Cm = 1 + 50 * theta, np.full(len(theta), 50.0), np.ones(T.shape)
    y, cen = simulate_ph(S, s, N, seed=DATA_KEY, censor_frac=cf)
    zexp = P.zexp_for(y)
    meths = ["ECS", "UNIF", "MHRS"] + (["DCS"] if cf > 0 else [])
    for meth, mode in [(m, md) for m in meths for md in ("host", "resident")]:
        if want & set(P.METHODS) and meth not in want:
            continue
        mm = P.METHODS[meth]
        sw = P.Sweeper(n, mm, 1)
        sw.set_obs(y, cen)
        run = sw.gibbs_resident if mode == "resident" else sw.gibbs
        P.set_seed(1)
        w = run(3, mm, nu, zeta, T, Cm, zexp)
        t0 = time.perf_counter()
        r = run(steps + 1, mm, nu, zeta, T, Cm, zexp, start=w[-1])
        dt = time.perf_counter() - t0
        ok = bool(np.all(np.isfinite(r))) and sw.flagged_obs == 0
        print(json.dumps({"config": name, "n": n, "N": N, "method": meth, "mode": mode, "steps": steps,
                          "sweeps_per_s": steps / dt, "ms_per_step": dt / steps * 1e3,
                          "kernel_ms_per_step": sw.kernel_ms_total / steps, "ok": ok}), flush=True)
        sw.close()
