"""CPU: the oracle pinned against the reference.

tests/golden/*.npz were produced by the reference's own C (oracle/_ref, built
from /root/reference/src, see tools/make_golden.py).  Bar: the restatement's
"ref" variant (R stream + libm) reproduces them bit for bit.  Where
oracle/_ref is present, the reference is re-run as well, so the fixtures
themselves are re-validated and the restatement is also checked on fresh
random cases (tests/test_oracle_ref.py).
"""
import os

import numpy as np
import pytest

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _load(name):
    return np.load(os.path.join(GOLD, name + ".npz"))


@pytest.mark.parametrize("tag", ["phtMCMC2", "phtMCMC"])
def test_g1_test_scripts_restatement(orc, tag):
    """tests/phtMCMC2.R and tests/phtMCMC.R, as .C vectors."""
    d = _load("g1_test_scripts")
    orc.set_seed(int(d[f"{tag}_seed"]))
    got = orc.gibbs(0, int(d[f"{tag}_it"]), int(d[f"{tag}_mhit"]), int(d[f"{tag}_method"]), int(d[f"{tag}_n"]),
                    d[f"{tag}_nu"], d[f"{tag}_zeta"], d[f"{tag}_T"], np.ones(16), d["x"])
    assert np.array_equal(got, d[f"{tag}_res"])


def test_g1_first_row_is_prior_mean():
    """Row 0 of the phtMCMC2 test chain is the prior-mean start nu/zeta
    (src/PHT_MCMC_Aslett.c:212-224): (24/16, 180/16)."""
    d = _load("g1_test_scripts")
    assert np.array_equal(d["phtMCMC2_res"][0], [1.4375, 11.1875])


@pytest.mark.parametrize("method", [2, 1])
def test_g2_cfg1_restatement(orc, method):
    """Config 1: n=3, N=200, 1000 sweeps (ECS and MHRS), every draw."""
    d = _load("g2_cfg1")
    orc.set_seed(int(d[f"m{method}_seed"]))
    got = orc.gibbs(0, int(d["it"]), 1, method, int(d["n"]), d["nu"], d["zeta"], d["T"], np.ones(16), d["y"])
    assert np.array_equal(got, d[f"m{method}_res"])


G3 = [(n, method, mhit) for n in (3, 4, 10) for method, mhit in ((1, 1), (1, 5), (2, 1), (4, 1))]


@pytest.mark.parametrize("n,method,mhit", G3)
def test_g3_per_observation_restatement(orc, n, method, mhit):
    """One step-1 sweep, per observation: start state, z and N identical."""
    d = _load("g3_sweeps")
    k = f"n{n}_m{method}_h{mhit}"
    orc.set_seed(int(d[k + "_seed"]))
    o = orc.ref_sweep(method, d[f"n{n}_S"], d[f"n{n}_s"], d[f"n{n}_y"], d[f"n{n}_cen"], mhit=mhit, per_obs=True)
    assert np.array_equal(o["B"], d[k + "_B"])
    assert np.array_equal(o["z"], d[k + "_z"])
    assert np.array_equal(o["N"], d[k + "_N"].astype(np.int32))
    # G4: the RNG consumption of every observation (MT words drawn)
    assert np.array_equal(o["nword"], d[k + "_nw"])


@pytest.mark.parametrize("n,method,mhit", G3[:4] + G3[8:])
def test_g3_reference_reproduces_fixture(ref, n, method, mhit):
    d = _load("g3_sweeps")
    k = f"n{n}_m{method}_h{mhit}"
    ref.set_seed(int(d[k + "_seed"]))
    nw = np.zeros(len(d[f"n{n}_y"]), np.uint32)
    B, z, N = ref.sweep(method, d[f"n{n}_S"], d[f"n{n}_s"], d[f"n{n}_y"], d[f"n{n}_cen"], mhit=mhit, nword=nw)
    assert np.array_equal(B, d[k + "_B"]) and np.array_equal(z, d[k + "_z"])
    assert np.array_equal(N, d[k + "_N"].astype(np.int32))
    assert np.array_equal(nw, d[k + "_nw"])


def test_g1_reference_reproduces_fixture(ref):
    d = _load("g1_test_scripts")
    for tag in ("phtMCMC2", "phtMCMC"):
        ref.set_seed(int(d[f"{tag}_seed"]))
        got = ref.gibbs(int(d[f"{tag}_it"]), 1, int(d[f"{tag}_method"]), 3, d[f"{tag}_nu"], d[f"{tag}_zeta"],
                        d[f"{tag}_T"], np.ones(16), d["x"])
        assert np.array_equal(got, d[f"{tag}_res"])
