"""GPU: statistical parity with the reference's algorithm at BASELINE.json's
full sizes.

One GPU step 1 over the whole configuration against the oracle's "ref"
variant (the reference's per-observation loop draw for draw,
src/Simulate_AbsCTMC_eq_Aslett_ECS.c:461-479,
src/Simulate_AbsCTMC_eq_Bladt_MHRS.c:63-114,
src/Simulate_AbsCTMC_eq_AslettHobolth_DCS.c:92-147) on the same (S, s, y):

* cfg2: BD-exit n = 5, N = 10^4 exact observations, ECS;
* cfg3: BD-exit n = 20, N = 10^5 exact observations, ECS (the n = 20 kernels:
  rows for the longest paths, a 13-point LDS envelope);
* cfg4: BD-exit n = 10, N = 10^6 exact observations, ECS (bench.py's data);
* cfg5: BD-exit n = 15, N = 5*10^5, 30 % censored; MHRS, DCS and ECS.

The two sides draw from different streams, so every cell of the sufficient
statistics (z_k and N_jk per observation) must agree in mean within
5 standard errors (oracle/posterior.py ``sweep_zscores``; per-observation
variances from both sides, the Poisson floor for rare transition cells).
The GPU's per-observation values come from the debug launch; the product
launch (``Sweeper.sweep``, no per-observation output) must return exactly
their totals.  With PHT_PARITY_REPORT=<file> each case appends its
resolution (the smallest per-cell bias the bar detects, 5 se, absolute and
relative to the cell mean) as one JSON line; DESIGN.md §2 quotes them.
"""
import json
import os

import numpy as np
import pytest

import phasetype_amd as P
from oracle import posterior as PO
from phasetype_amd.synth import DATA_KEY, bd_exit, simulate_ph

pytestmark = pytest.mark.gpu

# name -> (n, N, censored fraction, method)
CASES = {
    "cfg2_ecs": (5, 10_000, 0.0, 2),
    "cfg3_ecs": (20, 100_000, 0.0, 2),
    "cfg4_ecs": (10, 1_000_000, 0.0, 2),
    "cfg5_mhrs": (15, 500_000, 0.3, 1),
    "cfg5_dcs": (15, 500_000, 0.3, 4),
    "cfg5_ecs": (15, 500_000, 0.3, 2),
}
_DATA = {}


def _data(n, N, cf):
    k = (n, N, cf)
    if k not in _DATA:
        _DATA.clear()
        _DATA[k] = simulate_ph(*bd_exit(n), N, seed=DATA_KEY, censor_frac=cf)
    return _DATA[k]


def _report(name, zs, n, N, capped):
    path = os.environ.get("PHT_PARITY_REPORT")
    if not path:
        return
    zdet = PO.K_SIGMA * zs["z_se"]
    zrel = zdet / np.maximum(np.abs(zs["z_mean"]), 1e-300)
    live = zs["N_mean"] > 0
    ndet = PO.K_SIGMA * zs["N_se"]
    rec = dict(case=name, n=n, N=N, mhrs_capped_obs=capped, worst_z=float(zs["z"].max()), worst_N=float(zs["N"].max()),
               z_detectable_abs_max=float(zdet.max()), z_detectable_rel_median=float(np.median(zrel)),
               z_detectable_rel_max=float(zrel.max()),
               N_detectable_rel_median=float(np.median(ndet[live] / zs["N_mean"][live])),
               N_detectable_abs_max=float(ndet.max()))
    with open(path, "a") as f:
        f.write(json.dumps(rec) + "\n")


@pytest.mark.parametrize("name", list(CASES))
def test_full_size_sweep_statistics_vs_reference_algorithm(gpu, orc, name):
    n, N, cf, method = CASES[name]
    S, s = bd_exit(n)
    y, cen = _data(n, N, cf)
    zexp = P.zexp_for(y)
    orc.set_seed(0xF00 + method)
    r = orc.ref_sweep(method, S, s, y, cen)
    sw = P.Sweeper(n, method)
    sw.set_obs(y, cen)
    key = (0x51, 0x5EED + method)
    tot = sw.sweep(S, s, key=key, sweep=1, zexp=zexp)
    g = sw.sweep_debug(S, s, key=key, sweep=1, zexp=zexp)
    sw.close()
    k = 2 * n + n * n
    assert np.array_equal(tot[:k], g["stats"][:k]), "product launch differs from the per-observation launch"
    assert np.array_equal(g["zq"].sum(0), tot[:n])
    assert np.array_equal(g["N"].sum(0, dtype=np.int64), P.split_stats(tot, n)[2])
    # DESIGN.md §3 Caps: MHRS stops an observation after 2^22 rejected
    # attempts (survival to y below ~2.4e-7) and contributes its last attempt,
    # where the reference loops on; at cfg5 one observation of 5*10^5 (y =
    # 25.06) reaches it.  Its weight in a cell mean is <= y/N = 5e-5, far
    # below the bar's resolution.  Every other flag is a failure.
    fl = g["flags"]
    capped = int(np.count_nonzero(fl))
    assert np.all((fl == 0) | (fl == 16)) and capped <= 3, (np.unique(fl), capped)
    zs = PO.sweep_zscores(r["z"], r["N"], g["zq"] * 2.0 ** -zexp, g["N"])
    _report(name, zs, n, N, capped)
    assert zs["z"].max() < PO.K_SIGMA, (name, np.round(zs["z"], 2))
    assert zs["N"].max() < PO.K_SIGMA, (name, np.round(zs["N"], 2))
