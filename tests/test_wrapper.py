"""CPU: the Python mirror of the R wrappers (R/phtMCMC.R, R/phtMCMC2.R).

The wrappers only build the 15 .C vectors of LJMA_Gibbs and reshape ``res``.
Here LJMA_Gibbs is replaced (monkeypatch, test-only) by the oracle's "ref"
restatement, so the reference's own test scripts (tests/phtMCMC.R,
tests/phtMCMC2.R) run end to end on the CPU and must reproduce the golden
chains made by the reference's C (tests/golden/g1_test_scripts.npz).
"""
import os

import numpy as np
import pytest

import phasetype_amd as P

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


@pytest.fixture
def routed(monkeypatch, orc):
    calls = []

    def fake(it, mhit, method, n, m, nu, zeta, T, C_, y, l, censored, start, silent, res):
        Tf = np.asarray(T, np.int32).reshape(-1, order="F")
        Cf = np.asarray(C_, np.float64).reshape(-1, order="F")
        calls.append(dict(it=it, mhit=mhit, method=method, n=n, m=m, nu=list(nu), zeta=list(zeta), T=Tf, C=Cf,
                          l=l, censored=np.asarray(censored), start=list(start), silent=silent))
        out = orc.gibbs(0, it, mhit, method, n, nu, zeta, Tf, Cf, y, np.asarray(censored, np.int32),
                        np.asarray(start, np.float64))
        return {"res": out.T.reshape(-1).copy()}

    monkeypatch.setattr(P, "LJMA_Gibbs", fake)
    return calls


def test_phtMCMC2_test_script(routed, orc):
    """tests/phtMCMC2.R: set.seed(34752076); phtMCMC2(x, TT, dirpi, nu, zeta, 20)."""
    g = np.load(os.path.join(GOLD, "g1_test_scripts.npz"))
    TT = np.array(["0", "R", "R", "0", "F", "0", "0", "0", "F", "0", "0", "0", "0", "F", "F", "0"],
                  dtype=object).reshape(4, 4, order="F")
    orc.set_seed(34752076)
    out = P.phtMCMC2(g["x"], TT, [1, 0, 0], {"R": 180, "F": 24}, {"R": 16, "F": 16}, 20)
    c = routed[0]
    assert (c["it"], c["mhit"], c["method"], c["n"], c["m"]) == (20, 1, 2, 3, 2)
    assert c["nu"] == [24.0, 180.0] and c["zeta"] == [16.0, 16.0]  # order F, R
    assert list(c["T"]) == [0, 2, 2, 0, 1, 0, 0, 0, 1, 0, 0, 0, 0, 1, 1, 0]
    assert c["start"] == [-1.0] and c["l"] == 20 and not c["censored"].any()
    assert out["vars"] == ["F", "R"]
    assert np.array_equal(out["samples"], g["phtMCMC2_res"])


def test_phtMCMC_test_script(routed, orc):
    """tests/phtMCMC.R: set.seed(576734884); phtMCMC(x, 3, dirpi, nu, zeta, 6, mhit=1)."""
    g = np.load(os.path.join(GOLD, "g1_test_scripts.npz"))
    orc.set_seed(576734884)
    out = P.phtMCMC(g["x"], 3, [1, 0, 0], [24, 24, 1, 180, 1, 24, 180, 1, 24], [16, 16, 16], 6, mhit=1)
    c = routed[0]
    assert c["method"] == 1 and c["m"] == 9
    assert out["vars"] == ["S12", "S13", "S21", "S23", "S31", "S32", "s1", "s2", "s3"]  # C-locale sort
    assert c["nu"] == list(g["phtMCMC_nu"]) and list(c["T"]) == list(g["phtMCMC_T"])
    assert np.array_equal(out["samples"], g["phtMCMC_res"])


def test_phtMCMC_en_US_collation_order(routed, orc):
    g = np.load(os.path.join(GOLD, "g1_test_scripts.npz"))
    out = P.phtMCMC(g["x"], 3, [1, 0, 0], [24, 24, 1, 180, 1, 24, 180, 1, 24], [16, 16, 16], 2, collation="en_US")
    assert out["vars"] == ["s1", "S12", "S13", "s2", "S21", "S23", "s3", "S31", "S32"]
    # nu follows the names: s1 -> 1, S12 -> 24, ...
    assert routed[0]["nu"] == [1.0, 24.0, 24.0, 24.0, 180.0, 1.0, 24.0, 180.0, 1.0]


def test_phtMCMC_zeta_each_quirk(routed):
    """zeta is expanded rep(each=states+1) but named over the n^2 parameters
    (R/phtMCMC.R:29-30): row-specific values shift for rows >= 2."""
    x = np.array([0.5, 1.0, 2.0])
    P.phtMCMC(x, 3, [1, 0, 0], [1] * 9, [1.0, 2.0, 3.0], 2)
    # names in c(t(TT)) order: S12 S13 s1 | S21 S23 s2 | S31 S32 s3, zeta rep each 4: 1 1 1 1 2 2 2 2 3
    want = dict(zip(["S12", "S13", "s1", "S21", "S23", "s2", "S31", "S32", "s3"], [1, 1, 1, 1, 2, 2, 2, 2, 3]))
    order = ["S12", "S13", "S21", "S23", "S31", "S32", "s1", "s2", "s3"]
    assert routed[0]["zeta"] == [float(want[k]) for k in order]


def test_phtMCMC2_resume(routed, orc):
    g = np.load(os.path.join(GOLD, "g1_test_scripts.npz"))
    TT = np.array([["0", "F", "0", "0"], ["R", "0", "F", "0"], ["R", "0", "0", "F"], ["0", "0", "0", "0"]],
                  dtype=object)
    first = P.phtMCMC2(g["x"], TT, [1, 0, 0], {"R": 180, "F": 24}, {"R": 16, "F": 16}, 5)
    more = P.phtMCMC2(g["x"], TT, [1, 0, 0], {"R": 180, "F": 24}, {"R": 16, "F": 16}, 3, resume=first["samples"])
    assert routed[1]["start"] == list(first["samples"][-1]) and routed[1]["it"] == 4
    assert more["samples"].shape == (8, 2)
    assert np.array_equal(more["samples"][:5], first["samples"])


@pytest.mark.parametrize("method,code", [("ECS", 2), ("MHRS", 1), ("DCS", 4), (["MHRS", "DCS"], 5)])
def test_phtMCMC2_method_bitmask(routed, method, code):
    TT = np.array([["0", "a", "0"], ["b", "0", "c"], ["0", "0", "0"]], dtype=object)
    P.phtMCMC2([0.5, 1.0], TT, [1, 0], {"a": 1, "b": 1, "c": 1}, {"a": 1, "b": 1, "c": 1}, 2, method=method)
    assert routed[0]["method"] == code


@pytest.mark.parametrize("bad,err", [
    (dict(n=0), "invalid number of MCMC"),
    (dict(mhit=-1), "Metropolis-Hastings"),
    (dict(beta=[1]), "beta should be a vector"),
    (dict(beta=[-1, 1]), "Dirichlet"),
    (dict(method="XYZ"), "unknown sampling methods"),
    (dict(nu={"a": 1, "b": 1}), "prior nu"),
    (dict(C_=np.ones((2, 2))), "dimension of C"),
])
def test_phtMCMC2_argument_errors(routed, bad, err):
    TT = np.array([["0", "a", "0"], ["b", "0", "c"], ["0", "0", "0"]], dtype=object)
    kw = dict(x=[0.5, 1.0], TT=TT, beta=[1, 0], nu={"a": 1, "b": 1, "c": 1}, zeta={"a": 1, "b": 1, "c": 1}, n=2)
    kw.update(bad)
    with pytest.raises(ValueError, match=err):
        P.phtMCMC2(**kw)
    assert not routed


def test_phtMCMC2_structure_errors(routed):
    with pytest.raises(ValueError, match="diagonal"):
        P.phtMCMC2([1.0], np.array([["a", "b"], ["0", "0"]], dtype=object), [1], {"a": 1, "b": 1},
                   {"a": 1, "b": 1}, 2)
    with pytest.raises(ValueError, match="absorbing"):
        P.phtMCMC2([1.0], np.array([["0", "b"], ["c", "0"]], dtype=object), [1], {"b": 1, "c": 1},
                   {"b": 1, "c": 1}, 2)
