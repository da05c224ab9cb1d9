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


def test_reference_summaries_are_complete():
    d = np.load(GOLD)
    for name, case in PO.CASES.items():
        s = PO.unpack(d, name)
        m = 3 * case[0] - 2  # BD-exit: m = 3n - 2 parameters
        assert s["mean"].shape == (m,) and np.all(s["mean"] > 0)
        assert int(s["sweeps"]) >= 0.85 * case[-1]
        for st in PO.STATS:
            assert np.all(s[st + "_se"] > 0) and np.all(np.isfinite(s[st]))
