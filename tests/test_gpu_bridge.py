"""GPU: the bridge modes (PHT_MHRS=bridge, PHT_DCS=bridge; pht_unif.h ulaw 1/2).

MHRS's path law (the first successful rejection attempt of
LJMA_samplechain_Bladt, then mhit independence-MH steps,
src/Simulate_AbsCTMC_eq_Bladt_MHRS.c:63-114) and DCS's (end state
b ~ (pi e^{yS})_b s_b, the endpoint-conditioned path, censored observations
treated as exact, src/Simulate_AbsCTMC_eq_AslettHobolth_DCS.c:92-147) are
sampled exactly by the uniformisation kernels: no rejection attempts, no
eigensystem.  Checks, as for every sampler:

* bit for bit against the oracle's device specification (orc_set_bridge):
  per observation, whole chains (host loop, device-resident), several chains
  per launch;
* in distribution against the reference's algorithm ("ref" variant): per
  cell of one sweep at BASELINE's full sizes, chain-level posteriors of
  tests/golden/g5_posterior.npz, and the power pair (mhit = 1 vs 5).
"""
import os

import numpy as np
import pytest

import phasetype_amd as P
from oracle import posterior as PO
from phasetype_amd.synth import DATA_KEY, bd_exit, bd_exit_structure, simulate_ph

pytestmark = pytest.mark.gpu

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "g5_posterior.npz")
ENV = {1: "PHT_MHRS", 4: "PHT_DCS"}


@pytest.fixture
def bridge(monkeypatch, orc):
    """bridge(method): the device (env, read at context creation) and the
    oracle's dev variant both in bridge mode for that method"""
    def on(method):
        monkeypatch.setenv(ENV[method], "bridge")
        orc.set_bridge(mhrs=method == 1, dcs=method == 4)
    yield on
    orc.set_bridge(False, False)


def _perturbed(n, seed):
    S, s = bd_exit(n)
    rng = np.random.default_rng(seed)
    S = S.copy()
    mask = S > 0
    S[mask] *= rng.uniform(0.7, 1.3, mask.sum())
    s = s * rng.uniform(0.7, 1.3, n)
    np.fill_diagonal(S, 0.0)
    np.fill_diagonal(S, -(S.sum(1) + s))
    return S, s


def _cyclic_some_exits(n, seed=0):
    """complex spectrum, and states without an exit (s_j = 0): MHRS's law
    excludes them at y (the reference's re-draw loop)"""
    rng = np.random.default_rng(seed)
    S = np.zeros((n, n))
    for i in range(n):
        S[i, (i + 1) % n] = rng.uniform(1.5, 3.0)
        S[i, (i - 1) % n] += rng.uniform(0.0, 0.2)
    s = rng.uniform(0.1, 0.5, n)
    s[1::2] = 0.0
    np.fill_diagonal(S, 0.0)
    np.fill_diagonal(S, -(S.sum(1) + s))
    return S, s


@pytest.mark.parametrize("method,mhit,n,N,cf,gen", [(1, 1, 3, 3000, 0.3, "bd"), (1, 3, 10, 3000, 0.3, "bd"),
                                                    (1, 1, 15, 1500, 0.0, "bd"), (1, 2, 6, 2000, 0.3, "cyc"),
                                                    (4, 1, 4, 3000, 0.3, "bd"), (4, 1, 15, 1500, 0.3, "bd"),
                                                    (4, 1, 20, 1000, 0.0, "bd"), (4, 1, 6, 2000, 0.3, "cyc")])
def test_bridge_per_observation_bitexact(gpu, orc, bridge, method, mhit, n, N, cf, gen):
    bridge(method)
    S0, s0 = bd_exit(n)
    y, cen = simulate_ph(S0, s0, N, seed=6000 + n, censor_frac=cf)
    S, s = _perturbed(n, n + 5) if gen == "bd" else _cyclic_some_exits(n)
    key, sweep = (0x61 + n, 0x3), 2
    zexp = int(orc.lib.orc_zexp(np.ascontiguousarray(y), len(y)))
    o = orc.dev_sweep(method, S, s, y, cen, mhit=mhit, key=key, sweep=sweep, zexp=zexp)
    sw = P.Sweeper(n, method, mhit)
    sw.set_obs(y, cen)
    g = sw.sweep_debug(S, s, key=key, sweep=sweep, zexp=zexp)
    for f in ("B", "pre", "flags", "ndraw"):
        bad = np.nonzero(g[f] != o[f])[0]
        assert bad.size == 0, f"{f} differs at obs {bad[:5]}: gpu {g[f][bad[:5]]} oracle {o[f][bad[:5]]}"
    assert np.array_equal(g["zq"], o["zq"]) and np.array_equal(g["N"], o["N"])
    st = sw.sweep(S, s, key=key, sweep=sweep, zexp=zexp)
    sw.close()
    assert np.array_equal(st[:2 * n + n * n], g["stats"][:2 * n + n * n])
    assert not o["flags"].any()
    if gen == "cyc" and method == 1:
        ex = cen == 0
        assert np.all(s[o["pre"][ex]] > 0)  # the exact paths end in states with an exit


@pytest.mark.parametrize("method,mhit,cf", [(1, 1, 0.3), (1, 4, 0.0), (4, 1, 0.3)])
def test_bridge_chain_bitexact(gpu, orc, bridge, method, mhit, cf):
    """pht_gibbs_run, the .C LJMA_Gibbs and the device-resident chain in
    bridge mode == the oracle's chains (dev 1, dev 2)."""
    bridge(method)
    n = 5
    T, theta = bd_exit_structure(n)
    S, s = bd_exit(n)
    y, cen = simulate_ph(S, s, 3000, seed=71, censor_frac=cf)
    m, it = len(theta), 12
    nu, zeta, Cm = 1 + 50 * theta, np.full(m, 50.0), np.ones(T.shape)
    Tf, Cf = T.reshape(-1, order="F"), Cm.reshape(-1, order="F")
    zexp = P.zexp_for(y)
    for dev in (1, 2):
        orc.set_seed(5)
        want = orc.gibbs(dev, it, mhit, method, n, nu, zeta, Tf, Cf, y, cen)
        P.set_seed(5)
        sw = P.Sweeper(n, method, mhit)
        sw.set_obs(y, cen)
        got = sw.gibbs(it, method, nu, zeta, T, Cm, zexp) if dev == 1 else \
            sw.gibbs_resident(it, method, nu, zeta, T, Cm, zexp)
        sw.close()
        assert np.array_equal(got, want), dev
    orc.set_seed(6)
    want = orc.gibbs(1, it, mhit, method, n, nu, zeta, Tf, Cf, y, cen)
    P.set_seed(6)
    out = P.LJMA_Gibbs(it, mhit, method, n, m, nu, zeta, T, Cm, y, len(y), cen, [-1.0], 1, np.zeros(it * m))
    assert np.array_equal(out["res"].reshape(m, it).T, want)


@pytest.mark.parametrize("method", [1, 4])
def test_bridge_chains_one_launch(gpu, bridge, method):
    """several bridge chains per launch == the single runs"""
    bridge(method)
    n = 4
    T, theta = bd_exit_structure(n)
    S, s = bd_exit(n)
    y, cen = simulate_ph(S, s, 2000, seed=8, censor_frac=0.3)
    m = len(theta)
    nu, zeta, Cm = 1 + 50 * theta, np.full(m, 50.0), np.ones(T.shape)
    seeds = np.array([3, 4, 5], np.uint32)
    got, _ = P.gibbs_chains(seeds, y, cen, n, method, nu, zeta, T, Cm, mhit=2, it=6)
    for c, sd in enumerate(seeds):
        P.set_seed(int(sd))
        sw = P.Sweeper(n, method, 2)
        sw.set_obs(y, cen)
        want = sw.gibbs(6, method, nu, zeta, T, Cm, P.zexp_for(y))
        sw.close()
        assert np.array_equal(got[c], want), c


@pytest.mark.parametrize("name", ["cfg1_mhrs", "n15_cens_mhrs", "n4_y05_mhrs1", "n4_y05_mhrs5", "n15_cens_dcs"])
def test_bridge_chain_matches_reference_posterior(gpu, bridge, name):
    n, method, mhit, y, cen, T, nu, zeta = PO.case_inputs(name)
    bridge(method)
    ref = PO.unpack(np.load(GOLD), name)
    sw = P.Sweeper(n, method, mhit)
    sw.set_obs(y, cen)
    P.set_seed(4242)
    chain = sw.gibbs(9001, method, nu, zeta, T, np.ones(T.shape), P.zexp_for(y))
    sw.close()
    ok, worst, bad = PO.compare(PO.summarize(chain), ref)
    assert ok, (name, worst, bad[:5])
    assert sw.flagged_obs == 0


def test_bridge_chain_tells_mhrs_mhit_apart(gpu, bridge):
    """power: the bridge MHRS chain at mhit = 1 must fail the reference's
    mhit = 5 posterior (SURVEY.md §4.3's bias)"""
    n, method, mhit, y, cen, T, nu, zeta = PO.case_inputs("n4_y05_mhrs1")
    bridge(method)
    other = PO.unpack(np.load(GOLD), "n4_y05_mhrs5")
    sw = P.Sweeper(n, method, 1)
    sw.set_obs(y, cen)
    P.set_seed(4243)
    chain = sw.gibbs(9001, method, nu, zeta, T, np.ones(T.shape), P.zexp_for(y))
    sw.close()
    ok, worst, _ = PO.compare(PO.summarize(chain), other)
    assert not ok and worst > 8.0, worst


@pytest.mark.parametrize("name,n,N,cf,method", [("cfg4_mhrs", 10, 1_000_000, 0.0, 1),
                                                 ("cfg5_mhrs", 15, 500_000, 0.3, 1),
                                                 ("cfg5_dcs", 15, 500_000, 0.3, 4)])
def test_bridge_full_size_sweep_vs_reference_algorithm(gpu, orc, bridge, name, n, N, cf, method):
    """one bridge sweep over the whole BASELINE configuration against the
    reference's algorithm on the same (S, s, y): every cell within 5 se"""
    S, s = bd_exit(n)
    y, cen = simulate_ph(S, s, N, seed=DATA_KEY, censor_frac=cf)
    orc.set_seed(0xB00 + method)
    r = orc.ref_sweep(method, S, s, y, cen)
    bridge(method)
    zexp = P.zexp_for(y)
    sw = P.Sweeper(n, method)
    sw.set_obs(y, cen)
    g = sw.sweep_debug(S, s, key=(0x52, method), sweep=1, zexp=zexp)
    sw.close()
    assert not g["flags"].any()
    zs = PO.sweep_zscores(r["z"], r["N"], g["zq"] * 2.0 ** -zexp, g["N"])
    assert zs["z"].max() < PO.K_SIGMA, (name, np.round(zs["z"], 2))
    assert zs["N"].max() < PO.K_SIGMA, (name, np.round(zs["N"], 2))
