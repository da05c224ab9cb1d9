"""GPU parity beyond birth-death structure: the HIP kernels against the
oracle's device-spec restatement (ORC_DEV), bit for bit, per observation, on
generators whose shape the BD-exit cases never reach.

- "acyclic": upper-triangular sub-generators (Coxian-like; the general
  acyclic PH class): up to n - 1 successors per state, so moveMass' categorical
  (src/Simulate_AbsCTMC_eq_Aslett_ECS.c:350-358), the MHRS jump scan
  (src/Simulate_AbsCTMC_gt_Bladt_MHRS.c:49-121) and HobCDF's successor sums
  (src/Simulate_AbsCTMC_gt_Hobolth_DCS.c:74-226) run over long candidate
  lists; the spectrum is the (distinct) diagonal, so every state has an
  eigenvalue equal to its own S_jj and HobCDF/J take the reference's equal-
  eigenvalue branch (src/Simulate_AbsCTMC_gt_Hobolth_DCS.c:27,139).
- "reversible": dense generators with pi_i S_ij = pi_j S_ji (real spectrum,
  similar to a symmetric matrix), every state a successor of every other.
- "neareq": acyclic with two total rates equal to 1e-9 relative: the
  eigenvector matrix is nearly singular and DCS divides by 1e-9-relative
  differences just outside that branch's 1e-13 switch.

Data are simulated from the structure itself; the sweep runs at a perturbed
parameter (as a Gibbs sweep would).  ECS is also forced through the 16-lane
rows (PHT_ROWK).  Bar: B, pre, flags, draws consumed, fixed-point z and N
identical per observation, and the statistics block identical."""
import numpy as np
import pytest

import phasetype_amd as P
from phasetype_amd.synth import simulate_ph

pytestmark = pytest.mark.gpu


def acyclic(n, seed, neareq=False):
    rng = np.random.default_rng(seed)
    S = np.triu(rng.exponential(1.0, (n, n)) * (rng.random((n, n)) < 0.7), 1)
    for i in range(n - 1):  # every state can move on: the path can reach state n
        S[i, i + 1] = max(S[i, i + 1], 0.5)
    s = rng.exponential(0.4, n)
    s[-1] = 1.5
    rate = S.sum(1) + s + 0.21 * np.arange(n)  # distinct total rates
    if neareq:
        rate[n // 2] = rate[n // 2 - 1] * (1.0 + 1e-9)
    s = rate - S.sum(1)
    np.fill_diagonal(S, -rate)
    return S, s


def reversible(n, seed):
    rng = np.random.default_rng(seed)
    W = rng.uniform(0.2, 1.0, (n, n))
    W = (W + W.T) / 2.0
    pi = rng.dirichlet(np.ones(n))
    S = W * pi[None, :]  # pi_i S_ij = pi_i pi_j W_ij: symmetric
    np.fill_diagonal(S, 0.0)
    S *= 3.0 / S.sum(1).mean()
    s = rng.uniform(0.1, 0.6, n)
    np.fill_diagonal(S, -(S.sum(1) + s))
    return S, s


def perturb(S, s, seed):
    """Rates scaled by a symmetric random factor (keeps a reversible
    generator reversible, so its spectrum stays real)."""
    rng = np.random.default_rng(seed)
    F = rng.uniform(0.8, 1.25, S.shape)
    S = S * np.sqrt(F * F.T)
    s = s * rng.uniform(0.8, 1.25, len(s))
    np.fill_diagonal(S, 0.0)
    np.fill_diagonal(S, -(S.sum(1) + s))
    return S, s


def generator(kind, n, seed):
    if kind == "reversible":
        return reversible(n, seed)
    return acyclic(n, seed, neareq=(kind == "neareq"))


def neareq(S, s):
    """Total rates of states n/2 - 1 and n/2 equal to 1e-9 relative (through
    the exit rate of state n/2)."""
    S, s = S.copy(), s.copy()
    k = S.shape[0] // 2
    want = -S[k - 1, k - 1] * (1.0 + 1e-9)
    s[k] += want + S[k, k]
    S[k, k] = -want
    return S, s


def sweep_params(kind, S0, s0, seed):
    S, s = perturb(S0, s0, seed)
    return neareq(S, s) if kind == "neareq" else (S, s)


CASES = [
    # (kind, n, N, censored fraction, method)
    ("acyclic", 4, 4000, 0.3, 2), ("acyclic", 4, 3000, 0.3, 1), ("acyclic", 4, 3000, 0.3, 4),
    ("acyclic", 8, 3000, 0.3, 2), ("acyclic", 8, 2000, 0.3, 1), ("acyclic", 8, 2000, 0.0, 4),
    ("acyclic", 12, 2000, 0.3, 2), ("acyclic", 12, 1500, 0.3, 4), ("acyclic", 16, 1500, 0.0, 2),
    ("acyclic", 10, 3000, 0.3, 8), ("acyclic", 20, 1000, 0.3, 2),
    ("reversible", 5, 1500, 0.3, 2), ("reversible", 5, 800, 0.3, 1), ("reversible", 5, 1000, 0.3, 4),
    ("reversible", 10, 800, 0.3, 2), ("reversible", 10, 500, 0.0, 1), ("reversible", 10, 600, 0.3, 4),
    ("reversible", 15, 400, 0.3, 8),
    ("neareq", 6, 3000, 0.3, 2), ("neareq", 6, 2000, 0.3, 4), ("neareq", 6, 2000, 0.0, 1),
]


def _compare(g, o, N, n):
    for f in ("B", "pre", "flags", "ndraw"):
        bad = np.nonzero(g[f] != o[f])[0]
        assert bad.size == 0, f"{f} differs at obs {bad[:5]}: gpu {g[f][bad[:5]]} oracle {o[f][bad[:5]]}"
    bad = np.nonzero(np.any(g["zq"] != o["zq"], axis=1))[0]
    assert bad.size == 0, f"zq differs at obs {bad[:5]}"
    bad = np.nonzero(np.any(g["N"] != o["N"], axis=(1, 2)))[0]
    assert bad.size == 0, f"N differs at obs {bad[:5]}"
    zq, B, Nt, ex = P.split_stats(g["stats"], n)
    assert np.array_equal(zq, o["zq_tot"]) and np.array_equal(B, o["B_tot"]) and np.array_equal(Nt, o["N_tot"])
    assert ex[0] == N


@pytest.mark.parametrize("kind,n,N,cf,method", CASES)
def test_structure_per_observation_bitexact(gpu, orc, kind, n, N, cf, method):
    S0, s0 = generator(kind, n, 100 + n)
    y, cen = simulate_ph(S0, s0, N, seed=5000 + n, censor_frac=cf)
    S, s = sweep_params(kind, S0, s0, 7 * n + 1)
    key, sweep = (0x2468 + n, 0x1357), 3
    zexp = int(orc.lib.orc_zexp(np.ascontiguousarray(y), len(y)))
    o = orc.dev_sweep(method, S, s, y, cen, key=key, sweep=sweep, zexp=zexp)
    sw = P.Sweeper(n, method, 1)
    sw.set_obs(y, cen)
    g = sw.sweep_debug(S, s, key=key, sweep=sweep, zexp=zexp)
    _compare(g, o, N, n)
    st = sw.sweep(S, s, key=key, sweep=sweep, zexp=zexp)
    assert np.array_equal(st[:2 * n + n * n], g["stats"][:2 * n + n * n])


@pytest.mark.parametrize("kind,n", [("acyclic", 8), ("reversible", 10), ("acyclic", 20)])
def test_structure_rows_bitexact(gpu, orc, monkeypatch, kind, n):
    """ECS with every exact observation on a 16-lane row (pht_ecs_row.h):
    moveMass over up to n - 1 successors from the row's registers."""
    monkeypatch.setenv("PHT_ROWK", str(10 ** 9))
    S0, s0 = generator(kind, n, 200 + n)
    y, cen = simulate_ph(S0, s0, 1000, seed=6000 + n, censor_frac=0.2)
    S, s = sweep_params(kind, S0, s0, 3 * n)
    zexp = int(orc.lib.orc_zexp(np.ascontiguousarray(y), len(y)))
    o = orc.dev_sweep(2, S, s, y, cen, key=(21, 22), sweep=9, zexp=zexp)
    sw = P.Sweeper(n, 2, 1)
    sw.set_obs(y, cen)
    g = sw.sweep_debug(S, s, key=(21, 22), sweep=9, zexp=zexp)
    _compare(g, o, len(y), n)
