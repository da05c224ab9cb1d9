"""GPU: the device-resident Gibbs chain (pht_gibbs_run_resident; SURVEY.md
§8f.1-2, opt-in, non-parity): sweeps, conjugate Gamma updates and parameter
blocks all on the device, one host wait per run.

* bit for bit against the oracle's restatement of the same chain (oracle
  gibbs dev=2: the GPU spec's sweeps + include/pht_gamma.h draws +
  include/pht_eigen.h's eigensystem for ECS/DCS), every sampler, with
  censoring;
* in distribution against the reference: posterior means and quantiles
  within 5 combined MCSEs of tests/golden/g5_posterior.npz (ECS, DCS and
  MHRS against the reference's chains of the same sampler; UNIF against the
  reference's ECS chains — the same conditional path law);
* the guards: a method other than the context's, a complex spectrum (the
  device eigensystem stops the run), the processed-count check.
"""
import os

import numpy as np
import pytest

import phasetype_amd as P
from oracle import posterior as PO
from phasetype_amd.synth import bd_exit, bd_exit_structure, simulate_ph

pytestmark = pytest.mark.gpu

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "g5_posterior.npz")


@pytest.mark.parametrize("method,n,mhit,cf", [(8, 6, 1, 0.3), (8, 10, 1, 0.0), (1, 4, 1, 0.3), (1, 4, 3, 0.0),
                                              (8, 15, 1, 0.3), (2, 3, 1, 0.0), (2, 6, 1, 0.3), (2, 10, 1, 0.0),
                                              (2, 20, 1, 0.0), (4, 5, 1, 0.3), (4, 10, 1, 0.0)])
def test_resident_chain_bitexact(gpu, orc, method, n, mhit, cf):
    T, theta = bd_exit_structure(n)
    S, s = bd_exit(n)
    y, cen = simulate_ph(S, s, 3000, seed=21 + n, censor_frac=cf)
    m, it = len(theta), 25
    nu, zeta = 1 + 50 * theta, np.full(m, 50.0)
    Cm = np.ones_like(T, dtype=np.float64)
    orc.set_seed(123)
    want = orc.gibbs(2, it, mhit, method, n, nu, zeta, T.reshape(-1, order="F"), Cm.reshape(-1, order="F"), y, cen)
    P.set_seed(123)
    sw = P.Sweeper(n, method, mhit)
    sw.set_obs(y, cen)
    got = sw.gibbs_resident(it, method, nu, zeta, T, Cm, P.zexp_for(y))
    assert np.array_equal(got, want), np.abs(got - want).max()
    P.set_seed(123)
    again = sw.gibbs_resident(it, method, nu, zeta, T, Cm, P.zexp_for(y))
    assert np.array_equal(got, again)
    sw.close()


def test_resident_start_and_small_prior_shapes(gpu, orc):
    """A user start row; and priors with nu <= 1 (drawn, not the mode)."""
    n, method = 5, 8
    T, theta = bd_exit_structure(n)
    S, s = bd_exit(n)
    y, cen = simulate_ph(S, s, 2000, seed=3)
    m, it = len(theta), 8
    Cm = np.ones_like(T, dtype=np.float64)
    for nu, zeta, start in ((1 + 50 * theta, np.full(m, 50.0), theta * 1.2),
                            (np.full(m, 0.8), np.full(m, 0.5), None)):
        orc.set_seed(9)
        want = orc.gibbs(2, it, 1, method, n, nu, zeta, T.reshape(-1, order="F"), Cm.reshape(-1, order="F"), y, cen,
                         start=start)
        P.set_seed(9)
        sw = P.Sweeper(n, method, 1)
        sw.set_obs(y, cen)
        got = sw.gibbs_resident(it, method, nu, zeta, T, Cm, P.zexp_for(y), start=start)
        sw.close()
        assert np.array_equal(got, want)


@pytest.mark.parametrize("name,method", [("n10_ecs", 8), ("n15_cens_ecs", 8), ("n20_ecs", 8), ("cfg1_mhrs", 1),
                                         ("n15_cens_mhrs", 1), ("cfg1_ecs", 2), ("n10_ecs", 2),
                                         ("n15_cens_ecs", 2), ("n15_cens_dcs", 4)])
def test_resident_chain_matches_reference_posterior(gpu, name, method):
    n, _, mhit, y, cen, T, nu, zeta = PO.case_inputs(name)
    ref = PO.unpack(np.load(GOLD), name)
    sw = P.Sweeper(n, method, mhit)
    sw.set_obs(y, cen)
    P.set_seed(1618)
    chain = sw.gibbs_resident(9001, method, nu, zeta, T, np.ones(T.shape), P.zexp_for(y))
    sw.close()
    ok, worst, bad = PO.compare(PO.summarize(chain), ref)
    assert ok, (name, worst, bad[:5])
    assert sw.flagged_obs == 0


def test_resident_guards(gpu):
    n = 4
    T, theta = bd_exit_structure(n)
    S, s = bd_exit(n)
    y, cen = simulate_ph(S, s, 1000, seed=4)
    m = len(theta)
    nu, zeta, Cm = 1 + 50 * theta, np.full(m, 50.0), np.ones(T.shape)
    sw = P.Sweeper(n, 2, 1)
    sw.set_obs(y, cen)
    with pytest.raises(P.PhaseTypeError, match="context created for that method"):
        sw.gibbs_resident(5, 8, nu, zeta, T, Cm, P.zexp_for(y))
    sw.close()
    # a 3-cycle with weak exits: complex eigenvalues, the device eigensystem
    # stops the chain (the host path warns and uses the real parts)
    Tc = np.zeros((4, 4), np.int32)
    Tc[0, 1], Tc[1, 2], Tc[2, 0], Tc[0, 3], Tc[1, 3], Tc[2, 3] = 1, 1, 1, 2, 2, 2
    yc = np.random.default_rng(2).exponential(3.0, 500)
    sw = P.Sweeper(3, 2, 1)
    sw.set_obs(yc, np.zeros(500, np.int32))
    with pytest.raises(P.PhaseTypeError, match="eigensystem failed"):
        sw.gibbs_resident(4, 2, np.array([501.0, 6.0]), np.array([50.0, 50.0]), Tc, np.ones((4, 4)), P.zexp_for(yc))
    sw.close()
    sw = P.Sweeper(n, 8, 1)
    sw.set_obs(y, cen)
    sw.set_global_count(len(y) + 5)
    with pytest.raises(P.PhaseTypeError, match="did not sample every observation"):
        sw.gibbs_resident(5, 8, nu, zeta, T, Cm, P.zexp_for(y))
    sw.close()


def test_unif_cap_is_an_error(gpu):
    """UNIF observations the uniformisation table cannot sample exactly (rows
    beyond its capacity, or mu*y > 1300) carry a path that is not a draw of
    the target law (pht_unif.h): both loops fail the run instead of warning.
    Resident: the table is sized from the start (twice its largest exit
    rate, 2.8 -> 498 rows for y = 40); a strong prior at 10x the start's
    rates pulls the chain's rates (and the rows y = 40 needs) past it within
    a few sweeps.  The host loop sizes every sweep's table from its own
    rates, so the same run is fine there; it fails on one observation with
    mu*y > 1300."""
    n = 4
    T, theta = bd_exit_structure(n)
    S, s = bd_exit(n)
    y, cen = simulate_ph(S, s, 200, seed=5)
    y[0] = 40.0
    m = len(theta)
    nu, zeta, Cm = 1 + 5000 * theta, np.full(m, 500.0), np.ones(T.shape)
    sw = P.Sweeper(n, 8, 1)
    sw.set_obs(y, cen)
    with pytest.raises(P.PhaseTypeError, match="UNIF observations needed more"):
        sw.gibbs_resident(40, 8, nu, zeta, T, Cm, P.zexp_for(y), start=theta)
    P.set_seed(3)
    ok = sw.gibbs(40, 8, nu, zeta, T, Cm, P.zexp_for(y), start=theta)
    assert np.all(np.isfinite(ok)) and sw.flagged_obs == 0
    assert ok[-1].max() > 5 * theta.max()  # the rates did move far past the start
    sw.close()
    yb = y.copy()
    yb[1] = 1300.0 / 2.8 + 50.0  # mu = 2.8 for BD-exit(4) at the prior mode: lam > 1300
    sw = P.Sweeper(n, 8, 1)
    sw.set_obs(yb, cen)
    with pytest.raises(P.PhaseTypeError, match="UNIF observations need more"):
        sw.gibbs(3, 8, 1 + 50 * theta, np.full(m, 50.0), T, Cm, P.zexp_for(yb))
    sw.close()
