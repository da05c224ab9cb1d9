"""GPU: statistical parity of the HIP path with the reference's algorithm.

Parity with the reference itself is unpinned; its algorithm
is the restatement's "ref" variant (R stream, libm, the reference's
arithmetic order).  The GPU draws from a different random stream (Philox),
so it agrees with it in distribution:

* chain level: HIP Gibbs chains through
  pht_gibbs_run and through the .C entry point LJMA_Gibbs, summarised by
  per-parameter posterior means and 5/50/95 % quantiles, against the
  reference summaries of tests/golden/g5_posterior.npz, within 5 combined
  batch-means MCSEs per statistic (oracle/posterior.py): cfg1 ECS/MHRS,
  n = 10 ECS, n = 15 with 30 % censoring (MHRS, ECS, DCS), n = 20 ECS;
* sweep level: one GPU step 1 against the "ref" variant on the same
  (S, s, y), per-observation statistics within 5 standard errors, at
  n = 4, 10, 15, 20 with censoring.
"""
import os

import numpy as np
import pytest

import phasetype_amd as P
from oracle import posterior as PO
from phasetype_amd.synth import bd_exit, simulate_ph

pytestmark = pytest.mark.gpu

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "g5_posterior.npz")
GPU_SWEEPS = 9000


@pytest.mark.parametrize("name", list(PO.CASES))
def test_gpu_chain_matches_reference_posterior(gpu, name):
    n, method, mhit, y, cen, T, nu, zeta = PO.case_inputs(name)
    ref = PO.unpack(np.load(GOLD), name)
    sw = P.Sweeper(n, method, mhit)
    sw.set_obs(y, cen)
    P.set_seed(31337)
    chain = sw.gibbs(GPU_SWEEPS + 1, method, nu, zeta, T, np.ones(T.shape), P.zexp_for(y))
    sw.close()
    ok, worst, bad = PO.compare(PO.summarize(chain), ref)
    assert ok, (name, worst, bad[:5])
    assert sw.flagged_obs == 0


@pytest.mark.parametrize("name", ["n10_ecs", "n15_cens_dcs"])
def test_ljma_gibbs_chain_matches_reference_posterior(gpu, name):
    """The drop-in .C routine (all visible GPUs) against the same bar."""
    n, method, mhit, y, cen, T, nu, zeta = PO.case_inputs(name)
    ref = PO.unpack(np.load(GOLD), name)
    m, it = len(nu), GPU_SWEEPS + 1
    P.set_seed(4711)
    out = P.LJMA_Gibbs(it, mhit, method, n, m, nu, zeta, T, np.ones(T.shape), y, len(y), cen, [-1.0], 1,
                       np.zeros(it * m))
    chain = out["res"].reshape(m, it).T
    ok, worst, bad = PO.compare(PO.summarize(chain), ref)
    assert ok, (name, worst, bad[:5])


@pytest.mark.parametrize("name", ["cfg1_ecs", "n10_ecs", "n15_cens_ecs", "n20_ecs"])
def test_unif_chain_matches_ecs_reference_posterior(gpu, name):
    """The uniformisation sampler (method 8, no reference counterpart)
    samples the same conditional path law as ECS, so its chain must match the
    reference ECS posterior of the same data within the same tolerance."""
    n, method, mhit, y, cen, T, nu, zeta = PO.case_inputs(name)
    assert method == 2
    ref = PO.unpack(np.load(GOLD), name)
    sw = P.Sweeper(n, 8, 1)
    sw.set_obs(y, cen)
    P.set_seed(2718)
    chain = sw.gibbs(GPU_SWEEPS + 1, 8, nu, zeta, T, np.ones(T.shape), P.zexp_for(y))
    sw.close()
    ok, worst, bad = PO.compare(PO.summarize(chain), ref)
    assert ok, (name, worst, bad[:5])
    assert sw.flagged_obs == 0


def test_gpu_chain_detects_shifted_data(gpu):
    """Power of the same comparison: data scaled by 1.1 must fail it."""
    n, method, mhit, y, cen, T, nu, zeta = PO.case_inputs("n10_ecs")
    ref = PO.unpack(np.load(GOLD), "n10_ecs")
    sw = P.Sweeper(n, method, mhit)
    sw.set_obs(y * 1.1, cen)
    P.set_seed(31337)
    chain = sw.gibbs(GPU_SWEEPS + 1, method, nu, zeta, T, np.ones(T.shape), P.zexp_for(y * 1.1))
    sw.close()
    ok, worst, _ = PO.compare(PO.summarize(chain), ref)
    assert not ok and worst > 8.0, worst


@pytest.mark.parametrize("mhit", [1, 5])
def test_gpu_chain_tells_mhrs_mhit_apart(gpu, mhit):
    """Power against a subtle reference effect: the GPU
    MHRS chain at mhit = k matches the reference's mhit = k posterior (the
    parametrised test above) and must FAIL the other one (y in [0.45, 0.55],
    where mhit = 1's fresh-current-path bias is large)."""
    name = f"n4_y05_mhrs{mhit}"
    n, method, mhit_, y, cen, T, nu, zeta = PO.case_inputs(name)
    other = PO.unpack(np.load(GOLD), f"n4_y05_mhrs{6 - mhit}")
    sw = P.Sweeper(n, method, mhit_)
    sw.set_obs(y, cen)
    P.set_seed(31337)
    chain = sw.gibbs(GPU_SWEEPS + 1, method, nu, zeta, T, np.ones(T.shape), P.zexp_for(y))
    sw.close()
    ok, worst, _ = PO.compare(PO.summarize(chain), other)
    assert not ok and worst > 8.0, worst


def _gpu_vs_ref_sweep(orc, n, method, y, cen, mhit=1, seed=99, key=(3, 4)):
    """z-scores of one GPU step 1 (per-observation debug launch) against the
    "ref" variant on the same (S, s, y)."""
    S, s = bd_exit(n)
    zexp = P.zexp_for(y)
    orc.set_seed(seed)
    r = orc.ref_sweep(method, S, s, y, cen, mhit=mhit)
    sw = P.Sweeper(n, method, mhit)
    sw.set_obs(y, cen)
    g = sw.sweep_debug(S, s, key=key, sweep=1, zexp=zexp)
    sw.close()
    assert not g["flags"].any()
    return PO.sweep_zscores(r["z"], r["N"], g["zq"] * 2.0 ** -zexp, g["N"])


@pytest.mark.parametrize("n,cf,N", [(4, 0.3, 20000), (10, 0.3, 12000), (15, 0.3, 6000), (20, 0.0, 4000)])
def test_sweep_statistics_vs_reference_algorithm(gpu, orc, n, cf, N):
    """GPU step 1 vs the "ref" variant on identical (S, s, y): per-observation
    z and N agree in mean within 5 standard errors (different streams), for
    MHRS, ECS and DCS.  (Full BASELINE sizes: test_gpu_fullsize.py.)"""
    S, s = bd_exit(n)
    y, cen = simulate_ph(S, s, N, seed=11 + n, censor_frac=cf)
    for method in (1, 2, 4):
        zs = _gpu_vs_ref_sweep(orc, n, method, y, cen, seed=99 + n, key=(3, 4 + n))
        assert zs["z"].max() < PO.K_SIGMA and zs["N"].max() < PO.K_SIGMA, (method, n, zs["z"], zs["N"])


def test_sweep_statistics_tell_mhrs_mhit_apart(gpu, orc):
    """Power of the sweep-level bar: the GPU's MHRS at mhit = 1 matches the
    reference's mhit = 1 and FAILS its mhit = 5 (SURVEY.md §4.3's bias,
    3.8e-2 in E[z] at y = 0.5); at mhit = 5 the other way round."""
    y, cen = PO.grid_obs(50000, 0.45, 0.55)
    for mhit_gpu in (1, 5):
        same = _gpu_vs_ref_sweep(orc, 4, 1, y, cen, mhit=mhit_gpu, seed=7 + mhit_gpu, key=(9, mhit_gpu))
        assert max(same["z"].max(), same["N"].max()) < PO.K_SIGMA, (mhit_gpu, same["z"], same["N"])
        S, s = bd_exit(4)
        orc.set_seed(17)
        r = orc.ref_sweep(1, S, s, y, cen, mhit=6 - mhit_gpu)
        sw = P.Sweeper(4, 1, mhit_gpu)
        sw.set_obs(y, cen)
        zexp = P.zexp_for(y)
        g = sw.sweep_debug(S, s, key=(9, mhit_gpu), sweep=1, zexp=zexp)
        sw.close()
        other = PO.sweep_zscores(r["z"], r["N"], g["zq"] * 2.0 ** -zexp, g["N"])
        assert max(other["z"].max(), other["N"].max()) > 3 * PO.K_SIGMA, (mhit_gpu, other["z"])
