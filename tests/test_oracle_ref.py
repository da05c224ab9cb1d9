"""CPU: the oracle's two variants against each other and against analytics.

Parity with the reference is UNPINNED: the reference needs R
and cannot be built here, and its tests hold no fixtures.  The checks that
stand in for a pin are RNG-free:

* Van Loan conditional expectations E[z | Y=y], E[N | Y=y] for exact
  observations, and their censored counterparts
  E[z | Y>y], E[N | Y>y] (matrix-exponential integrals, below), which the
  reference's samplers target: ECS and DCS exactly, MHRS as mhit grows, DCS
  treating censored observations as exact (src/Simulate_AbsCTMC_eq_
  AslettHobolth_DCS.c:132-133);
* the "dev" variant (the GPU specification: Philox stream, detmath exp/log,
  fixed-point z) against the "ref" variant (the reference's algorithm draw
  for draw, R stream + libm) in distribution, at the configs' state counts
  n = 4, 10, 15, 20 (5 standard errors per statistic).

Whole chains of the "ref" variant are pinned to their regression vectors in
tests/test_golden.py.
"""
import numpy as np
import pytest
from scipy.linalg import expm

from phasetype_amd.synth import bd_exit, bd_exit_structure, simulate_ph


def test_resume_start_vector(orc):
    """start[0] != -1 resumes from the given parameters (src/PHT_MCMC_Aslett.c:195-207):
    row 0 is the start, later rows are draws."""
    n = 3
    T, theta = bd_exit_structure(n)
    S, s = bd_exit(n)
    y, _ = simulate_ph(S, s, 100, seed=9)
    nu, zeta = 1 + 10 * theta, np.full(len(theta), 10.0)
    start = theta * 1.1
    orc.set_seed(5)
    got = orc.gibbs(0, 8, 1, 2, n, nu, zeta, T.reshape(-1, order="F"), np.ones(T.size), y, start=start)
    assert np.array_equal(got[0], start)
    assert np.all(np.isfinite(got)) and np.all(got[1:] > 0) and not np.array_equal(got[1], start)


# ---------------------------------------------------------------- statistics
def _mc_agree(a, b, k=5.0):
    """Means of two independent samples (rows = observations) agree within k s.e."""
    a, b = np.asarray(a, float), np.asarray(b, float)
    se = np.sqrt(a.var(0) / len(a) + b.var(0) / len(b))
    return np.abs(a.mean(0) - b.mean(0)) <= k * se + 1e-12


STAT_CASES = [(4, 2, 1, 0.3), (4, 1, 1, 0.3), (4, 1, 4, 0.0), (4, 4, 1, 0.3),
              (10, 2, 1, 0.0), (10, 1, 1, 0.0), (10, 4, 1, 0.0),
              (15, 2, 1, 0.3), (15, 1, 1, 0.3), (15, 4, 1, 0.3),
              (20, 2, 1, 0.0)]


@pytest.mark.parametrize("n,method,mhit,cf", STAT_CASES)
def test_dev_variant_matches_ref_variant_statistically(orc, n, method, mhit, cf):
    N = 20000 if n <= 10 else 8000
    S, s = bd_exit(n)
    y, cen = simulate_ph(S, s, N, seed=21 + n, censor_frac=cf)
    orc.set_seed(8)
    r = orc.ref_sweep(method, S, s, y, cen, mhit=mhit)
    o = orc.dev_sweep(method, S, s, y, cen, mhit=mhit, key=(11, 12 + n), sweep=1)
    zd = o["zq"] * 2.0 ** -o["zexp"]
    bad = ~_mc_agree(r["z"], zd)
    assert not bad.any(), (np.nonzero(bad), r["z"].mean(0), zd.mean(0))
    assert np.all(_mc_agree(r["N"].reshape(N, -1), o["N"].reshape(N, -1)))
    assert np.array_equal(np.bincount(o["B"], minlength=n)[1:], np.zeros(n - 1))  # pi = e1 (quirk q1)
    assert np.array_equal(np.bincount(r["B"], minlength=n)[1:], np.zeros(n - 1))
    assert not o["flags"].any() and not r["flags"].any()


def _van_loan(S, s, y):
    """E[z_i | Y=y], E[N_ij | Y=y] (j = n: absorption) for PH(e1, S)."""
    n = S.shape[0]
    pi = np.zeros(n)
    pi[0] = 1.0
    f = pi @ expm(S * y) @ s
    Ez, EN = np.zeros(n), np.zeros((n, n + 1))
    for i in range(n):
        for j in range(n):
            A = np.zeros((n, n))
            A[i, j] = 1.0
            M = np.block([[S, A], [np.zeros((n, n)), S]])
            J = pi @ expm(M * y)[:n, n:] @ s / f
            if i == j:
                Ez[i] = J
            else:
                EN[i, j] = S[i, j] * J
        EN[i, n] = (pi @ expm(S * y))[i] * s[i] / f
    return Ez, EN


def _van_loan_censored(S, s, y):
    """E[z_i | Y>y], E[N_ij | Y>y] for PH(e1, S): the part of the path before
    y by Van Loan blocks (end vector 1 = alive at y), the part after y by
    pi e^{yS} (-S)^{-1} e_i, the expected time in i after y."""
    n = S.shape[0]
    pi = np.zeros(n)
    pi[0] = 1.0
    one = np.ones(n)
    Ey = pi @ expm(S * y)
    surv = Ey @ one
    after = Ey @ np.linalg.inv(-S)  # expected time in each state after y
    Ez, EN = np.zeros(n), np.zeros((n, n + 1))
    for i in range(n):
        for j in range(n):
            A = np.zeros((n, n))
            A[i, j] = 1.0
            M = np.block([[S, A], [np.zeros((n, n)), S]])
            J = (pi @ expm(M * y)[:n, n:] @ one + (after[i] if i == j else 0.0)) / surv
            if i == j:
                Ez[i] = J
            else:
                EN[i, j] = S[i, j] * (J + after[i] / surv)
        EN[i, n] = after[i] * s[i] / surv
    return Ez, EN


def _check_expectations(o, n, Ez, EN, reps, tag, S):
    """Means within 5 s.e.; for rarely visited states and rare transitions the
    sample variance is floored at the Poisson one implied by the expectation
    (counts: var >= E; times: var >= E x the mean sojourn)."""
    z = o["zq"] * 2.0 ** -o["zexp"]
    var = np.maximum(z.var(0), np.abs(Ez) / -np.diag(S))
    assert np.all(np.abs(z.mean(0) - Ez) <= 5 * np.sqrt(var / reps) + 1e-9), (tag, z.mean(0), Ez)
    Nd = o["N"].astype(float)
    Nfull = np.concatenate([Nd * (1 - np.eye(n)), np.diagonal(Nd, axis1=1, axis2=2)[:, :, None]], axis=2)
    m, var = Nfull.mean(0), np.maximum(Nfull.var(0), np.abs(EN))
    assert np.all(np.abs(m - EN) <= 5 * np.sqrt(var / reps) + 1e-9), (tag, m, EN)


VL_CASES = [(4, 2, 1), (4, 4, 1), (4, 1, 25), (10, 2, 1), (10, 4, 1), (15, 2, 1), (15, 4, 1), (20, 2, 1)]


@pytest.mark.parametrize("n,method,mhit", VL_CASES)
def test_dev_variant_van_loan(orc, n, method, mhit):
    """Exact observations: dev-variant conditional means == Van Loan expectations
    (ECS and DCS are exact samplers; MHRS only as mhit grows)."""
    reps = 4000
    S, s = bd_exit(n)
    for yv in (0.5, 3.0) if n <= 4 else (2.0, 8.0):
        o = orc.dev_sweep(method, S, s, np.full(reps, yv), None, mhit=mhit, key=(99, int(yv * 10) + n), sweep=2)
        Ez, EN = _van_loan(S, s, yv)
        _check_expectations(o, n, Ez, EN, reps, (n, method, yv), S)


@pytest.mark.parametrize("n,method", [(4, 2), (4, 1), (10, 2), (10, 1), (15, 2)])
def test_dev_variant_censored_expectations(orc, n, method):
    """Censored observations (ECS via LJMA_samplechain, MHRS's rejection
    loop): conditional means == E[z | Y>y], E[N | Y>y] (SURVEY.md §4.3's
    censored probe, here analytic)."""
    reps = 4000
    S, s = bd_exit(n)
    for yv in (0.5, 3.0):
        o = orc.dev_sweep(method, S, s, np.full(reps, yv), np.ones(reps, np.int32), key=(98, int(yv * 10) + n),
                          sweep=3)
        Ez, EN = _van_loan_censored(S, s, yv)
        _check_expectations(o, n, Ez, EN, reps, (n, method, yv, "cens"), S)


def test_dcs_treats_censored_as_exact(orc):
    """DCS ignores the censoring flag (src/Simulate_AbsCTMC_eq_AslettHobolth_DCS.c:132-133):
    its censored-observation means are the exact-at-y expectations."""
    n, reps, yv = 4, 4000, 3.0
    S, s = bd_exit(n)
    o = orc.dev_sweep(4, S, s, np.full(reps, yv), np.ones(reps, np.int32), key=(97, 1), sweep=4)
    Ez, EN = _van_loan(S, s, yv)
    _check_expectations(o, n, Ez, EN, reps, "dcs-cens", S)


@pytest.mark.parametrize("n", [3, 5, 10, 15, 20])
def test_dcs_halley_root_matches_find02(orc, n):
    """The device spec's DCS jump-time root (hob_halley) against
    Find02's Brent search (the reference's root finder) on the same draws:
    every discrete outcome identical, z equal to the CDF evaluation's
    rounding, and 2.4-3.1x fewer CDF evaluations."""
    S, s = bd_exit(n)
    y, cen = simulate_ph(S, s, 2000, seed=70 + n, censor_frac=0.3)
    out = {}
    try:
        for brent in (True, False):
            orc.set_dcs_brent(brent)
            out[brent] = orc.dev_sweep(4, S, s, y, cen, key=(0xD5 + n, 3), sweep=2)
    finally:
        orc.set_dcs_brent(False)
    a, b = out[True], out[False]
    for f in ("B", "pre", "N", "ndraw", "flags"):
        assert np.array_equal(a[f], b[f]), f
    rel = np.abs(a["z"] - b["z"]).max() / np.abs(a["z"]).max()
    assert rel < 1e-9, rel
    assert a["stats"][1] > 2.2 * b["stats"][1], (a["stats"][1], b["stats"][1])


@pytest.mark.parametrize("n,cf", [(10, 0.0), (15, 0.3)])
def test_dcs_halley_wavefront_maximum(orc, n, cf):
    """A jump-converged DCS round waits for its slowest lane: the expected
    maximum over 64 lanes of the Halley root's evaluations per jump
    (tools/dcs_halley_hist.py).  r03's stop bound left ~3 % of jumps
    bisecting at the noise floor (E[max] ~9.9); r04's bound and log-survival
    first step bring it to ~4.7.  Guards both changes."""
    S, s = bd_exit(n)
    y, cen = simulate_ph(S, s, 6000, seed=90 + n, censor_frac=cf)
    orc.halley_hist()
    orc.dev_sweep(4, S, s, y, cen, key=(0xE1, n), sweep=1, per_obs=False)
    h = orc.halley_hist().astype(float)
    p = h / h.sum()
    cdf = np.cumsum(p)
    mean = float((np.arange(64) * p).sum())
    emax = float(sum(1.0 - cdf[k] ** 64 for k in range(64)))
    assert mean < 3.45 and emax < 5.0, (mean, emax)


def test_censored_expectations_by_forward_simulation():
    """The censored analytics above against brute-force forward simulation
    conditioned on Y > y (the survey's censored probe)."""
    n, yv = 4, 1.0
    S, s = bd_exit(n)
    Ez, EN = _van_loan_censored(S, s, yv)
    rng = np.random.default_rng(3)
    rates = -np.diag(S)
    P = np.zeros((n, n + 1))
    P[:, :n] = S / rates[:, None]
    P[np.arange(n), np.arange(n)] = 0.0
    P[:, n] = s / rates
    cum = np.cumsum(P, 1)
    M = 200000
    st = np.zeros(M, np.int64)
    t = np.zeros(M)
    z = np.zeros((M, n))
    Nc = np.zeros((M, n, n + 1))
    alive = np.ones(M, bool)
    while alive.any():
        idx = np.nonzero(alive)[0]
        d = rng.exponential(1.0, idx.size) / rates[st[idx]]
        z[idx, st[idx]] += d
        t[idx] += d
        nxt = (rng.random(idx.size)[:, None] > cum[st[idx]]).sum(1)
        Nc[idx, st[idx], nxt] += 1
        st[idx] = nxt
        alive[idx] = nxt < n
    keep = t > yv
    zk, Nk = z[keep], Nc[keep]
    se = zk.std(0) / np.sqrt(keep.sum())
    assert np.all(np.abs(zk.mean(0) - Ez) <= 5 * se), (zk.mean(0), Ez)
    seN = Nk.std(0) / np.sqrt(keep.sum())
    assert np.all(np.abs(Nk.mean(0) - EN) <= 5 * seN + 1e-9), (Nk.mean(0), EN)


# ------------------------------------------- the uniformisation sampler (UNIF)
def _cyclic(n, seed=0):
    """A generator with a complex spectrum: a cycle 0 -> 1 -> ... -> n-1 -> 0
    with exits and weak back-steps (the reference's ECS/DCS keep only the real
    parts of its eigenvalues, src/utility.c:118-120)."""
    rng = np.random.default_rng(seed)
    S = np.zeros((n, n))
    for i in range(n):
        S[i, (i + 1) % n] = rng.uniform(1.5, 3.0)
        S[i, (i - 1) % n] += rng.uniform(0.0, 0.2)
    s = rng.uniform(0.1, 0.5, n)
    np.fill_diagonal(S, 0.0)
    np.fill_diagonal(S, -(S.sum(1) + s))
    return S, s


@pytest.mark.parametrize("n,gen", [(4, "bd"), (10, "bd"), (20, "bd"), (5, "cyclic"), (12, "cyclic")])
def test_unif_van_loan(orc, n, gen):
    """UNIF (method 8, the uniformisation sampler of pht_unif.h) is an exact
    sampler of the conditional path law: its conditional means equal the
    Van Loan expectations for exact AND censored observations, also for
    generators with complex spectra (where eigen-based samplers fail)."""
    S, s = bd_exit(n) if gen == "bd" else _cyclic(n)
    if gen == "cyclic":
        assert np.abs(np.linalg.eigvals(S).imag).max() > 0.1  # really complex
    reps = 4000
    for yv in (0.5, 3.0, 8.0):
        for cens in (0, 1):
            o = orc.dev_sweep(8, S, s, np.full(reps, yv), np.full(reps, cens, np.int32), key=(7, n), sweep=9)
            assert not o["flags"].any()
            Ez, EN = (_van_loan_censored if cens else _van_loan)(S, s, yv)
            _check_expectations(o, n, Ez, EN, reps, (n, gen, yv, cens), S)


def test_unif_shard_and_order_invariance(orc):
    """An observation's UNIF result depends only on its own id, y and the
    parameters: a shard (obs0 offset, a different table length K from its
    own largest y) reproduces the full run's per-observation results."""
    n = 6
    S, s = bd_exit(n)
    y, cen = simulate_ph(S, s, 3000, seed=5, censor_frac=0.3)
    full = orc.dev_sweep(8, S, s, y, cen, key=(1, 2), sweep=3, zexp=40)
    part = orc.dev_sweep(8, S, s, y[1000:1100], cen[1000:1100], key=(1, 2), sweep=3, zexp=40, obs0=1000)
    for f in ("B", "pre", "zq", "N", "ndraw"):
        assert np.array_equal(full[f][1000:1100], part[f]), f


def test_unif_flags_extreme_lam(orc):
    """mu y beyond 1300 (the unnormalised Poisson weights would overflow) is
    a flagged cap, not a wrong draw."""
    S, s = bd_exit(3)
    o = orc.dev_sweep(8, S, s, np.array([1.0, 600.0]), np.zeros(2, np.int32), key=(1, 1), sweep=1, zexp=30)
    assert o["flags"][0] == 0 and o["flags"][1] & 64
