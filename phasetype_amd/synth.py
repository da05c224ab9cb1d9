"""Synthetic absorption-time data for tests and bench.py.

"BD-exit(n)": a birth-death phase-type generator with exits,
    S[i, i+1] = 2.0 (i < n-1), S[i, i-1] = 0.5 (i > 0),
    s_i = 0.3 (i < n-1), s_{n-1} = 2.0, S_ii = -(row sum),
every non-zero rate its own parameter (m = 3n - 2), pi = e_1.
Observations are y_i ~ PH(e_1, S) by forward simulation of the CTMC with a
seeded Philox generator; optional right-censoring replaces y_i by y_i * U_i
with probability `censor_frac` and sets censored_i = 1.
"""
from __future__ import annotations

import numpy as np

DATA_KEY = 0x50485431_20241008


def bd_exit(n: int, fwd: float = 2.0, back: float = 0.5, exit_: float = 0.3, last_exit: float = 2.0):
    """(S, s) of BD-exit(n): column-major-agnostic numpy (n,n), (n,)."""
    S = np.zeros((n, n))
    s = np.full(n, exit_)
    s[n - 1] = last_exit
    for i in range(n):
        if i + 1 < n:
            S[i, i + 1] = fwd
        if i > 0:
            S[i, i - 1] = back
    for i in range(n):
        S[i, i] = -(S[i].sum() + s[i])
    return S, s


def bd_exit_structure(n: int):
    """phtMCMC2-style structure: T (n+1)x(n+1) int parameter map (1-based,
    0 = structural zero), parameter truths theta[m] in T's index order."""
    S, s = bd_exit(n)
    G = np.zeros((n + 1, n + 1))
    G[:n, :n] = S
    G[:n, n] = s
    T = np.zeros((n + 1, n + 1), np.int32)
    theta = []
    for i in range(n):  # name order = row-major order of non-zero off-diagonals
        for j in range(n + 1):
            if i != j and G[i, j] > 0:
                theta.append(G[i, j])
                T[i, j] = len(theta)
    return T, np.array(theta)


def simulate_ph(S, s, N: int, seed: int = DATA_KEY, censor_frac: float = 0.0):
    """Forward-simulate N absorption times of PH(e_1, S); vectorised."""
    n = S.shape[0]
    rng = np.random.Generator(np.random.Philox(key=seed))
    rates = -np.diag(S)
    P = np.zeros((n, n + 1))
    P[:, :n] = S / rates[:, None]
    P[np.arange(n), np.arange(n)] = 0.0
    P[:, n] = s / rates
    cum = np.cumsum(P, axis=1)
    cum[:, -1] = 1.0
    y = np.zeros(N)
    state = np.zeros(N, np.int64)
    alive = np.ones(N, bool)
    while alive.any():
        idx = np.nonzero(alive)[0]
        st = state[idx]
        y[idx] += rng.exponential(1.0, idx.size) / rates[st]
        u = rng.random(idx.size)
        nxt = (u[:, None] > cum[st]).sum(axis=1)
        state[idx] = nxt
        alive[idx] = nxt < n
    cens = np.zeros(N, np.int32)
    if censor_frac > 0:
        c = rng.random(N) < censor_frac
        y[c] *= rng.random(int(c.sum()))
        cens[c] = 1
    return y, cens
