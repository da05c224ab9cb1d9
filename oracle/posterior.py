"""oracle/posterior.py — TEST INFRASTRUCTURE ONLY: chain-level posterior parity.

SURVEY.md §4.4 item 4: long-chain posterior means and quantiles of the GPU
chain against chains of the reference's algorithm (the restatement's "ref"
variant: R stream, libm, the reference's arithmetic order; bit-exact with the
regression vectors of tests/golden/), within Monte Carlo standard error by
batch means.  The two chains use different random streams, so they agree only
in distribution: a chain is summarised by, per parameter, its mean and its
5/50/95 % quantiles, each with a batch-means MCSE, and two summaries agree
when every statistic differs by at most K_SIGMA combined MCSEs.

Tolerance (stated in DESIGN.md §2): |a - b| <= 5 sqrt(mcse_a^2 + mcse_b^2)
per statistic, 25 batches after a 10 % burn-in.  The chains start at the
prior mode, which is the data-generating truth (priors nu = 1 + 50 theta,
zeta = 50), so they are stationary from the start.

The cases (CASES) cover every sampler at the configs' state counts: cfg1's
ECS and MHRS (n = 3, N = 200: the G2 data), BD-exit n = 10 (ECS), n = 15
with 30 % censoring (MHRS, ECS, and DCS, which treats censored observations
as exact, src/Simulate_AbsCTMC_eq_AslettHobolth_DCS.c:132-133) and n = 20
(ECS).  tools/make_golden.py writes the reference summaries to
tests/golden/g5_posterior.npz; tests compare HIP chains (and the oracle's
device-spec chain) against them.
"""
from __future__ import annotations

import numpy as np

from phasetype_amd.synth import bd_exit, bd_exit_structure, simulate_ph

K_SIGMA = 5.0
NBATCH = 25
BURN = 0.1
QUANTS = (0.05, 0.5, 0.95)

# name -> (n, N, censored fraction, method bitmask, mhit, data seed, reference sweeps)
CASES = {
    "cfg1_ecs": (3, 200, 0.0, 2, 1, 0xC0F1, 4000),
    "cfg1_mhrs": (3, 200, 0.0, 1, 1, 0xC0F1, 4000),
    "n10_ecs": (10, 2000, 0.0, 2, 1, 0x510, 3000),
    "n15_cens_ecs": (15, 1500, 0.3, 2, 1, 0x515, 3000),
    "n15_cens_mhrs": (15, 1500, 0.3, 1, 1, 0x515, 3000),
    "n15_cens_dcs": (15, 1500, 0.3, 4, 1, 0x515, 3000),
    "n20_ecs": (20, 1000, 0.0, 2, 1, 0x520, 3000),
    # power pair: MHRS with mhit = 1 is biased (the
    # "current" path is a fresh rejection draw every sweep),
    # mhit = 5 much less so; on short observations (y on a grid in
    # [0.45, 0.55]) the two posteriors differ and the harness must tell them
    # apart (tests/test_posterior.py, tests/test_gpu_posterior.py)
    "n4_y05_mhrs1": (4, 2000, 0.0, 1, 1, 0, 3000),
    "n4_y05_mhrs5": (4, 2000, 0.0, 1, 5, 0, 3000),
}
# cases whose data is a deterministic grid instead of PH(e1, S) draws
GRID_DATA = {"n4_y05_mhrs1": (0.45, 0.55), "n4_y05_mhrs5": (0.45, 0.55)}


def grid_obs(N: int, lo: float, hi: float):
    """N exact observations evenly spread over (lo, hi)."""
    return lo + (hi - lo) * (np.arange(N) + 0.5) / N, np.zeros(N, np.int32)


def case_inputs(name):
    """(n, method, mhit, y, censored, T, nu, zeta) of a case; T as (n+1)^2 int."""
    n, N, cf, method, mhit, seed, _ = CASES[name]
    S, s = bd_exit(n)
    T, theta = bd_exit_structure(n)
    if name in GRID_DATA:
        y, cen = grid_obs(N, *GRID_DATA[name])
    else:
        y, cen = simulate_ph(S, s, N, seed=seed, censor_frac=cf)
    nu, zeta = 1.0 + 50.0 * theta, np.full(len(theta), 50.0)
    return n, method, mhit, y, cen, T, nu, zeta


def summarize(chain, nbatch: int = NBATCH, burn: float = BURN) -> dict:
    """Per-parameter mean and QUANTS quantiles of a chain [it, m] (row 0 =
    the start, dropped with the burn-in), each with a batch-means MCSE."""
    x = np.asarray(chain, np.float64)[1:]
    x = x[int(len(x) * burn):]
    L = len(x) // nbatch
    x = x[len(x) - L * nbatch:]
    b = x.reshape(nbatch, L, -1)
    out = {"mean": x.mean(0), "mean_se": b.mean(1).std(0, ddof=1) / np.sqrt(nbatch), "sweeps": np.int64(len(x))}
    for q in QUANTS:
        k = f"q{int(round(q * 100)):02d}"
        out[k] = np.quantile(x, q, axis=0)
        out[k + "_se"] = np.quantile(b, q, axis=1).std(0, ddof=1) / np.sqrt(nbatch)
    return out


STATS = ["mean"] + [f"q{int(round(q * 100)):02d}" for q in QUANTS]


def compare(a: dict, b: dict, k: float = K_SIGMA):
    """(ok, worst z-score, report of the failing statistics)."""
    bad, worst = [], 0.0
    for st in STATS:
        se = np.sqrt(a[st + "_se"] ** 2 + b[st + "_se"] ** 2) + 1e-300
        z = np.abs(a[st] - b[st]) / se
        worst = max(worst, float(z.max()))
        for i in np.nonzero(z > k)[0]:
            bad.append(f"{st}[{i}]: {a[st][i]:.6g} vs {b[st][i]:.6g} (z = {z[i]:.2f})")
    return not bad, worst, bad


def _cell_moments(X, chunk: int = 65536):
    """(mean, variance) per cell of per-observation arrays X [L, ...],
    accumulated in chunks (integer counts exactly, in int64)."""
    L = X.shape[0]
    integer = np.issubdtype(X.dtype, np.integer)
    s1 = s2 = None
    for i in range(0, L, chunk):
        x = np.ascontiguousarray(X[i:i + chunk]).reshape(min(chunk, L - i), -1)
        x = x.astype(np.int64 if integer else np.float64)
        a, b = x.sum(0), (x * x).sum(0)
        s1, s2 = (a, b) if s1 is None else (s1 + a, s2 + b)
    mean = s1 / L
    return mean, np.maximum(s2 / L - mean * mean, 0.0)


def sweep_zscores(za, Na, zb, Nb):
    """Per-cell agreement of two step-1 sweeps over the same observations
    (different random streams): |mean_a - mean_b| / se for every z_k (per
    observation sojourn totals) and every N_jk (transition counts, diagonal
    = absorptions), se = sqrt(var_a/L + var_b/L) from the per-observation
    variances, floored for N at the Poisson level of the pooled mean
    (sqrt((m_a + m_b)/L)) so rare cells are not over-weighted.  Returns
    dict(z, N: z-scores; z_se, N_se: the standard errors; z_mean, N_mean:
    side a's means).  The smallest per-cell bias the 5-sigma bar detects
    is 5 se."""
    L = za.shape[0]
    out = {}
    for key, A, B in (("z", za, zb), ("N", Na, Nb)):
        ma, va = _cell_moments(A)
        mb, vb = _cell_moments(B)
        se = np.sqrt(va / L + vb / L)
        if key == "N":
            se = np.maximum(se, np.sqrt((ma + mb) / L))
        d = np.abs(ma - mb)
        out[key] = np.where(se > 0, d / np.where(se > 0, se, 1.0), np.where(d > 0, np.inf, 0.0))
        out[key + "_se"], out[key + "_mean"] = se, ma
    return out


def pack(prefix: str, summ: dict) -> dict:
    return {f"{prefix}_{k}": v for k, v in summ.items()}


def unpack(d, prefix: str) -> dict:
    keys = ["mean", "mean_se", "sweeps"] + [s + suf for s in STATS[1:] for suf in ("", "_se")]
    return {k: d[f"{prefix}_{k}"] for k in keys}
