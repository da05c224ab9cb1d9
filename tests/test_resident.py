"""CPU: the device-resident chain's pieces in the oracle (SURVEY.md §8f.1-2;
opt-in, non-parity).

* The counter-based Gamma sampler (include/pht_gamma.h, shared by the HIP
  update kernel and the oracle) against scipy's Gamma law: Kolmogorov-
  Smirnov over shapes from 0.3 (the a < 1 boost) to 10^5, and the scale.
* The resident chain (oracle gibbs dev=2: device Gamma update; UNIF sweeps,
  and ECS sweeps on the resident eigensystem) against the reference ECS
  posterior of cfg1 (oracle/posterior.py): same data and priors, within 5
  combined MCSEs.
GPU: tests/test_gpu_resident.py (bit-exact with this oracle chain)."""
import os

import numpy as np
import pytest
from scipy import stats

from oracle import posterior as PO

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "g5_posterior.npz")


@pytest.mark.parametrize("a", [0.3, 0.9, 1.0, 2.5, 24.0, 180.0, 1e5])
def test_counter_gamma_law(orc, a):
    x = orc.rgamma_ctr(a, 1.0, 20000, key=(11, int(a * 10) & 0xFFFF))
    assert np.all(np.isfinite(x)) and np.all(x > 0)
    assert stats.kstest(x, stats.gamma(a).cdf).pvalue > 1e-4
    y = orc.rgamma_ctr(a, 0.25, 2000, key=(11, int(a * 10) & 0xFFFF))
    assert np.allclose(y, 0.25 * x[:2000], rtol=1e-15, atol=0)  # same stream, scaled


def test_counter_gamma_is_deterministic_and_keyed(orc):
    a = orc.rgamma_ctr(3.0, 1.0, 100, key=(1, 2))
    assert np.array_equal(a, orc.rgamma_ctr(3.0, 1.0, 100, key=(1, 2)))
    assert not np.array_equal(a, orc.rgamma_ctr(3.0, 1.0, 100, key=(1, 3)))


@pytest.mark.parametrize("name,method", [("cfg1_ecs", 8), ("cfg1_ecs", 2)])
def test_resident_chain_matches_reference_posterior(orc, name, method):
    """UNIF, and ECS with the resident eigensystem (include/pht_eigen.h)."""
    n, _, mhit, y, cen, T, nu, zeta = PO.case_inputs(name)
    orc.set_seed(5)
    chain = orc.gibbs(2, 3001, 1, method, n, nu, zeta, T.reshape(-1, order="F"), np.ones(T.size), y, cen)
    ok, worst, bad = PO.compare(PO.summarize(chain), PO.unpack(np.load(GOLD), name))
    assert ok, (worst, bad[:5])
