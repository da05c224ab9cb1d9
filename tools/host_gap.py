#!/usr/bin/env python3
"""Per-sweep host cost on the GPU box: pht_build_params alone (dgeevx + the
packed block) per n, and a whole Gibbs sweep with a tiny shard (N = 64 exact
observations: the kernel is ~µs, so ms per sweep ~ the fixed host + launch +
copy + wait cost).  usage (GPU box): python3 tools/host_gap.py"""
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import phasetype_amd as P  # noqa: E402
from phasetype_amd.synth import DATA_KEY, bd_exit, bd_exit_structure, simulate_ph  # noqa: E402

L = P.load()
out = {}
for n in (5, 10, 15, 20):
    S, s = bd_exit(n)
    Sf = np.ascontiguousarray(S.ravel(order="F"))
    sc = np.ascontiguousarray(s)
    nb = L.pht_params_bytes(n)
    buf = np.zeros(nb, np.uint8)
    for _ in range(200):
        L.pht_build_params(n, Sf, sc, 2, buf.ctypes.data, nb)
    K = 3000
    t = time.perf_counter()
    for _ in range(K):
        L.pht_build_params(n, Sf, sc, 2, buf.ctypes.data, nb)
    out[f"build_params_us_n{n}"] = (time.perf_counter() - t) / K * 1e6
    T, theta = bd_exit_structure(n)
    nu, zeta = 1.0 + 50.0 * theta, np.full(len(theta), 50.0)
    y, cen = simulate_ph(S, s, 64, seed=DATA_KEY)
    sw = P.Sweeper(n, 2, 1)
    sw.set_obs(y, cen)
    zexp = P.zexp_for(y)
    P.set_seed(1)
    sw.gibbs(20, 2, nu, zeta, T, np.ones(T.shape), zexp)
    it = 400
    t = time.perf_counter()
    sw.gibbs(it + 1, 2, nu, zeta, T, np.ones(T.shape), zexp)
    dt = time.perf_counter() - t
    out[f"sweep_us_n{n}_N64"] = dt / it * 1e6
    out[f"kernel_us_n{n}_N64"] = sw.kernel_ms_total / it * 1e3
    sw.close()
print(json.dumps(out, indent=1))
