#!/usr/bin/env python3
"""Why a fresh MHRS chain's first ~100 sweeps cost more than its steady state
(VERDICT r04 weak 5 / next 5).

MHRS (src/Simulate_AbsCTMC_gt_Bladt_MHRS.c:49-121) repeats forward attempts
until one is alive at y (exact observation) with s[pre] > 0, so observation
i costs ~1/p_i(theta) attempts, p_i(theta) = pi e^{y_i S} 1[s > 0]; with
mhit = 1 there are two such searches per exact observation (the "current"
path and the proposal, src/Simulate_AbsCTMC_eq_Bladt_MHRS.c:63-101).  The
sum over 10^6 observations is dominated by the largest y, whose survival is
~ c e^{-|lambda_1| y} with lambda_1 the slowest decay rate of S.  The chain's
draw of S moves lambda_1, and the attempt count follows.

This script (GPU box) runs a cfg4-shaped MHRS chain (BD-exit n = 10,
N = 10^6, priors nu = 1 + 50 theta, zeta = 50, start at the prior mode =
the truth, as bench.py), then replays single sweeps at a subset of the
chain's parameter draws, recording per sweep: the kernel time, the uniforms
drawn (stats word 3, ~ attempts x jumps), the MHRS round counts, and the
analytic expected attempt count sum_i 2 / p_i(theta) with lambda_1.  One
JSON line per replayed sweep, then a summary line with the correlation of
kernel time against the expected attempt count.

usage: python3 tools/mhrs_burnin.py [--sweeps 400] [--every 10]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import phasetype_amd as P  # noqa: E402
from phasetype_amd.synth import DATA_KEY, bd_exit, bd_exit_structure, simulate_ph  # noqa: E402


def generator(theta, T, n):
    """(S, s) from the parameter vector through T (1-based, 0 = zero)."""
    G = np.zeros((n + 1, n + 1))
    m = T > 0
    G[m] = theta[T[m] - 1]
    S = G[:n, :n].copy()
    s = G[:n, n].copy()
    np.fill_diagonal(S, 0.0)
    np.fill_diagonal(S, -(S.sum(1) + s))
    return S, s


def expected_attempts(S, s, y):
    """sum_i (1 + mhit) / p_i with p_i = e_1 e^{y_i S} 1[s > 0] (exact obs)."""
    lam, V = np.linalg.eig(S)
    lam, V = lam.real, V.real
    c = np.linalg.solve(V, (s > 0).astype(float))  # e^{yS} w = V diag(e^{lam y}) V^-1 w
    a = V[0, :] * c
    p = np.exp(np.outer(y, lam)) @ a
    p = np.maximum(p, 1e-300)
    return float(np.sum(2.0 / p)), float(np.max(lam)), float(np.sum(2.0 / p[np.argsort(-y)[:1000]]))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sweeps", type=int, default=400)
    ap.add_argument("--every", type=int, default=10)
    ap.add_argument("--n", type=int, default=10)
    ap.add_argument("--N", type=int, default=1_000_000)
    ap.add_argument("--ab", default="", help="i,j: replay the draws of sweeps i and j alternately (30 pairs) instead")
    a = ap.parse_args()
    n = a.n
    S0, s0 = bd_exit(n)
    T, theta = bd_exit_structure(n)
    m = len(theta)
    nu, zeta = 1.0 + 50.0 * theta, np.full(m, 50.0)
    y, cen = simulate_ph(S0, s0, a.N, seed=DATA_KEY)
    zexp = P.zexp_for(y)
    sw = P.Sweeper(n, P.METHODS["MHRS"], 1)
    sw.set_obs(y, cen)
    P.set_seed(20241008)  # bench.py's seed: the same chain as the bench's warm-up + timed sweeps
    t0 = time.perf_counter()
    res = sw.gibbs(a.sweeps + 1, P.METHODS["MHRS"], nu, zeta, T, np.ones(T.shape), zexp)
    chain_s = time.perf_counter() - t0
    if a.ab:
        i, j = (int(v) for v in a.ab.split(","))
        gens = {i: generator(res[i], T, n), j: generator(res[j], T, n)}
        kt = {i: [], j: []}
        for rep in range(30):
            for it in (i, j):
                S, s = gens[it]
                st = sw.sweep(S, s, key=(11, 13 + rep), sweep=it + 1, zexp=zexp)
                kt[it].append(sw.last_kernel_ms())
        for it in (i, j):
            ea, lam1, _ = expected_attempts(*gens[it], y)
            print(json.dumps({"sweep": it, "kernel_ms_first5": kt[it][:5], "kernel_ms_median": float(np.median(kt[it])),
                              "expected_attempts": ea, "lambda1": lam1, "theta": [float(v) for v in res[it]]}),
                  flush=True)
        sw.close()
        return
    rows = []
    for it in range(0, a.sweeps + 1, a.every):
        S, s = generator(res[it], T, n)
        # replay: one sweep at this draw (3 repeats, median kernel time)
        ks, nd = [], 0
        for rep in range(3):
            st = sw.sweep(S, s, key=(11, 13 + rep), sweep=it + 1, zexp=zexp)
            ks.append(sw.last_kernel_ms())
            nd = int(P.split_stats(st, n)[3][3])
        ea, lam1, ea_top = expected_attempts(S, s, y)
        r = {"sweep": it, "kernel_ms": float(np.median(ks)), "uniforms": nd, "expected_attempts": ea,
             "expected_attempts_top1000": ea_top, "lambda1": lam1}
        rows.append(r)
        print(json.dumps(r), flush=True)
    k = np.array([r["kernel_ms"] for r in rows])
    e = np.array([r["expected_attempts"] for r in rows])
    u = np.array([r["uniforms"] for r in rows], float)
    first = [r for r in rows if 3 <= r["sweep"] <= 102]
    late = [r for r in rows if r["sweep"] > 200]
    print(json.dumps({
        "chain_sweeps": a.sweeps, "chain_s": chain_s,
        "corr_kernel_vs_expected_attempts": float(np.corrcoef(k, e)[0, 1]),
        "corr_kernel_vs_uniforms": float(np.corrcoef(k, u)[0, 1]),
        "kernel_ms_sweeps_3_102": float(np.mean([r["kernel_ms"] for r in first])) if first else None,
        "kernel_ms_after_200": float(np.mean([r["kernel_ms"] for r in late])) if late else None,
        "expected_attempts_3_102": float(np.mean([r["expected_attempts"] for r in first])) if first else None,
        "expected_attempts_after_200": float(np.mean([r["expected_attempts"] for r in late])) if late else None,
        "lambda1_truth": expected_attempts(S0, s0, y)[1], "expected_attempts_truth": expected_attempts(S0, s0, y)[0],
    }), flush=True)
    sw.close()


if __name__ == "__main__":
    main()
