"""CPU: the chain-level posterior harness (oracle/posterior.py, SURVEY.md
§4.4 item 4) on the oracle's device-specification chain.

tests/golden/g5_posterior.npz holds posterior summaries (mean and 5/50/95 %
quantiles per parameter, batch-means MCSEs) of long chains of the
reference's algorithm (the restatement's "ref" variant).  Here the device
variant (the GPU specification: Philox stream, detmath, fixed-point z) runs
its own chain on the same data and priors, and must agree within
5 combined MCSEs per statistic; the GPU chains face the same bar in
test_gpu_posterior.py.  The harness must also have power: a chain on data
scaled by 1.15 (a shifted posterior) must fail it.
"""
import os

import numpy as np
import pytest

from oracle import posterior as PO

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "g5_posterior.npz")


def _dev_chain(orc, name, it, scale=1.0, seed=11):
    n, method, mhit, y, cen, T, nu, zeta = PO.case_inputs(name)
    orc.set_seed(seed)
    return orc.gibbs(1, it + 1, mhit, method, n, nu, zeta, T.reshape(-1, order="F"), np.ones(T.size), y * scale,
                     cen)


@pytest.mark.parametrize("name", ["cfg1_ecs", "cfg1_mhrs"])
def test_device_spec_chain_matches_reference_posterior(orc, name):
    ref = PO.unpack(np.load(GOLD), name)
    got = PO.summarize(_dev_chain(orc, name, 2000))
    ok, worst, bad = PO.compare(got, ref)
    assert ok, (worst, bad[:5])


def test_harness_detects_a_shifted_posterior(orc):
    ref = PO.unpack(np.load(GOLD), "cfg1_mhrs")
    got = PO.summarize(_dev_chain(orc, "cfg1_mhrs", 2000, scale=1.15))
    ok, worst, _ = PO.compare(got, ref)
    assert not ok and worst > 8.0, worst


@pytest.mark.parametrize("mhit", [1, 5])
def test_chain_harness_tells_mhrs_mhit_apart(orc, mhit):
    """Power against a subtle reference effect: MHRS
    with mhit = 1 is biased.  The device-spec chain at
    mhit = k must match the reference's mhit = k posterior and fail the
    other one, on y in [0.45, 0.55]."""
    d = np.load(GOLD)
    got = PO.summarize(_dev_chain(orc, f"n4_y05_mhrs{mhit}", 2000))
    ok, worst, bad = PO.compare(got, PO.unpack(d, f"n4_y05_mhrs{mhit}"))
    assert ok, (worst, bad[:5])
    ok, worst, _ = PO.compare(got, PO.unpack(d, f"n4_y05_mhrs{6 - mhit}"))
    assert not ok and worst > 8.0, worst


def test_sweep_harness_tells_mhrs_mhit_apart(orc):
    """The per-cell sweep comparison (PO.sweep_zscores, used at full size in
    test_gpu_fullsize.py): the reference's MHRS at mhit = 1 against itself
    (another stream) and against the device spec passes; against mhit = 5 it
    fails (3.8e-2 in E[z] at y = 0.5)."""
    from phasetype_amd.synth import bd_exit

    S, s = bd_exit(4)
    y, cen = PO.grid_obs(30000, 0.45, 0.55)
    orc.set_seed(1)
    a = orc.ref_sweep(1, S, s, y, cen, mhit=1)
    orc.set_seed(2)
    b = orc.ref_sweep(1, S, s, y, cen, mhit=1)
    orc.set_seed(3)
    c = orc.ref_sweep(1, S, s, y, cen, mhit=5)
    dv = orc.dev_sweep(1, S, s, y, cen, mhit=1, key=(5, 6))
    zd = dv["zq"] * 2.0 ** -dv["zexp"]
    for other_z, other_N in ((b["z"], b["N"]), (zd, dv["N"])):
        zs = PO.sweep_zscores(a["z"], a["N"], other_z, other_N)
        assert max(zs["z"].max(), zs["N"].max()) < PO.K_SIGMA, (zs["z"], zs["N"])
    zs = PO.sweep_zscores(a["z"], a["N"], c["z"], c["N"])
    assert max(zs["z"].max(), zs["N"].max()) > 3 * PO.K_SIGMA


def test_reference_summaries_are_complete():
    d = np.load(GOLD)
    for name, case in PO.CASES.items():
        s = PO.unpack(d, name)
        m = 3 * case[0] - 2  # BD-exit: m = 3n - 2 parameters
        assert s["mean"].shape == (m,) and np.all(s["mean"] > 0)
        assert int(s["sweeps"]) >= 0.85 * case[-1]
        for st in PO.STATS:
            assert np.all(s[st + "_se"] > 0) and np.all(np.isfinite(s[st]))


@pytest.mark.parametrize("method,mhit,n,N,cf,grid", [(1, 1, 4, 30000, 0.0, True), (1, 5, 4, 30000, 0.0, True),
                                                     (1, 1, 10, 20000, 0.3, False), (4, 1, 10, 20000, 0.3, False)])
def test_bridge_device_spec_matches_reference_sweep(orc, method, mhit, n, N, cf, grid):
    """The bridge modes' device specification (PHT_MHRS=bridge /
    PHT_DCS=bridge: MHRS's / DCS's path law by uniformisation, pht_unif.h
    ulaw 1 / 2) against the reference's own sampler ("ref" variant) on the
    same (S, s, y), per cell within 5 se; the mhit = 1 grid case carries
    MHRS's fresh-current-path bias, which the bridge must reproduce."""
    from phasetype_amd.synth import bd_exit, simulate_ph

    S, s = bd_exit(n)
    y, cen = PO.grid_obs(N, 0.45, 0.55) if grid else simulate_ph(S, s, N, seed=3, censor_frac=cf)
    orc.set_seed(11)
    r = orc.ref_sweep(method, S, s, y, cen, mhit=mhit)
    orc.set_bridge(mhrs=method == 1, dcs=method == 4)
    try:
        d = orc.dev_sweep(method, S, s, y, cen, mhit=mhit, key=(3, 4))
    finally:
        orc.set_bridge(False, False)
    assert not d["flags"].any()
    zs = PO.sweep_zscores(r["z"], r["N"], d["zq"] * 2.0 ** -d["zexp"], d["N"])
    assert zs["z"].max() < PO.K_SIGMA and zs["N"].max() < PO.K_SIGMA, (zs["z"], zs["N"])
