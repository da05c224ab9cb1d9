#!/usr/bin/env python3
"""Generate tests/golden/*.npz from the CPU restatement's "ref" variant.

``python tools/make_golden.py``.  The fixtures hold inputs and outputs only.
They are REGRESSION vectors of the restatement (oracle/, "ref" variant: R's
stream + libm + the reference's arithmetic order), not pins: the reference
needs R's headers, nmath and RNG, which this image lacks, so it is unbuildable
here ("parity unpinned").  G1–G3 were first written in round 1
by a build of the reference against stand-in R headers; round 3 retired that
build and regenerates the same files from the restatement, bit for bit
(``--check`` compares without writing).  Per SURVEY.md §8(c):

* G1 ``g1_test_scripts.npz`` — LJMA_Gibbs chains of the reference's two test
  scripts, with the exact .C vectors of SURVEY.md §4.2 (tests/phtMCMC.R:1-22,
  tests/phtMCMC2.R:1-21; their 20 observations are the scripts' own data).
* G2 ``g2_cfg1.npz`` — config 1 (n=3 BD-exit, N=200 synthetic exact obs,
  1000 sweeps) for ECS and MHRS.
* G3 ``g3_sweeps.npz`` — one step-1 sweep, per observation (start state B,
  z, N), for n in {3, 4, 10}, 100 exact + 100 censored observations, methods
  MHRS (mhit 1 and 5), ECS, DCS, one R stream per case.
* G4 (keys ``*_nw`` of ``g3_sweeps.npz``) — the RNG consumption of each of
  those observations: 32-bit Mersenne-Twister words the reference drew
  (the draw-order check of Appendix A).

* G5 ``g5_posterior.npz`` — posterior summaries of long "ref"-variant chains
  (oracle/posterior.py CASES: cfg1 ECS/MHRS, n = 10 ECS, n = 15 with 30 %
  censoring MHRS/ECS/DCS, n = 20 ECS): per parameter the mean and the
  5/50/95 % quantiles with batch-means MCSEs.

usage: python3 tools/make_golden.py [--check] [g1_test_scripts g2_cfg1 g3_sweeps g5_posterior]
(no names: all fixtures)
"""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

from oracle import oracle as O  # noqa: E402
from phasetype_amd.synth import bd_exit, bd_exit_structure, simulate_ph  # noqa: E402

OUT = os.path.join(REPO, "tests", "golden")

# the 20 observations of tests/phtMCMC.R:6-10 and tests/phtMCMC2.R:6-10
X20 = np.array([
    1.45353415045187, 1.85349532001349, 2.01084961814576, 0.505725921290172,
    1.56252630012213, 3.41158665930278, 1.52674487509487, 4.3428662377235,
    8.03208018151311, 2.41746547476986, 0.38828086509283, 2.61513815012196,
    3.39148865480856, 1.82705817807965, 1.42090953713845, 0.851438991331866,
    0.0178808867191894, 0.632198596390046, 0.959910259815998, 1.83344199966323])

# .C vectors
PHTMCMC2_ARGS = dict(seed=34752076, it=20, mhit=1, method=2, n=3, nu=[24.0, 180.0], zeta=[16.0, 16.0],
                     T=[0, 2, 2, 0, 1, 0, 0, 0, 1, 0, 0, 0, 0, 1, 1, 0])
# phtMCMC: names sorted in the C locale: S12 S13 S21 S23 S31 S32 s1 s2 s3
#   T[i + 4 j] = index of the name at TT[i, j]
_names = ["S12", "S13", "S21", "S23", "S31", "S32", "s1", "s2", "s3"]
_nu_by = dict(zip(["S12", "S13", "s1", "S21", "S23", "s2", "S31", "S32", "s3"], [24, 24, 1, 180, 1, 24, 180, 1, 24]))
_T1 = np.zeros((4, 4), np.int32)
for i in range(3):
    for j in range(3):
        if i != j:
            _T1[i, j] = _names.index(f"S{i + 1}{j + 1}") + 1
    _T1[i, 3] = _names.index(f"s{i + 1}") + 1
PHTMCMC_ARGS = dict(seed=576734884, it=6, mhit=1, method=1, n=3, nu=[float(_nu_by[k]) for k in _names],
                    zeta=[16.0] * 9, T=list(_T1.reshape(-1, order="F")))


def perturbed(n, seed):
    S, s = bd_exit(n)
    rng = np.random.default_rng(seed)
    S = S.copy()
    mask = S > 0
    S[mask] *= rng.uniform(0.7, 1.3, mask.sum())
    s = s * rng.uniform(0.7, 1.3, n)
    np.fill_diagonal(S, 0.0)
    np.fill_diagonal(S, -(S.sum(1) + s))
    return S, s


def g1(orc):
    out = {"x": X20}
    for tag, a in (("phtMCMC2", PHTMCMC2_ARGS), ("phtMCMC", PHTMCMC_ARGS)):
        orc.set_seed(a["seed"])
        m = len(a["nu"])
        res = orc.gibbs(0, a["it"], a["mhit"], a["method"], a["n"], a["nu"], a["zeta"], np.array(a["T"], np.int32),
                        np.ones(16), X20, np.zeros(20, np.int32), np.array([-1.0]))
        out[f"{tag}_res"] = res
        for k in ("seed", "it", "mhit", "method", "n"):
            out[f"{tag}_{k}"] = np.int64(a[k])
        out[f"{tag}_nu"] = np.array(a["nu"])
        out[f"{tag}_zeta"] = np.array(a["zeta"])
        out[f"{tag}_T"] = np.array(a["T"], np.int32)
        assert res.shape == (a["it"], m)
    return out


def g2(orc):
    n, N, it = 3, 200, 1000
    S, s = bd_exit(n)
    T, theta = bd_exit_structure(n)
    y, cen = simulate_ph(S, s, N, seed=0xC0F1, censor_frac=0.0)
    nu, zeta = 1 + 50 * theta, np.full(len(theta), 50.0)
    out = {"y": y, "T": T.reshape(-1, order="F").astype(np.int32), "nu": nu, "zeta": zeta, "n": np.int64(n),
           "it": np.int64(it)}
    for method, seed in ((2, 101), (1, 102)):
        orc.set_seed(seed)
        out[f"m{method}_seed"] = np.int64(seed)
        out[f"m{method}_res"] = orc.gibbs(0, it, 1, method, n, nu, zeta, T.reshape(-1, order="F"), np.ones(T.size), y)
    return out


G3_CASES = [(n, method, mhit) for n in (3, 4, 10) for method, mhit in ((1, 1), (1, 5), (2, 1), (4, 1))]


def g3(orc):
    out = {}
    for n in (3, 4, 10):
        S0, s0 = bd_exit(n)
        ye, _ = simulate_ph(S0, s0, 100, seed=500 + n, censor_frac=0.0)
        yc, _ = simulate_ph(S0, s0, 100, seed=600 + n, censor_frac=0.0)
        rng = np.random.default_rng(700 + n)
        yc = yc * rng.uniform(0.05, 1.0, 100)  # right-censoring times
        y = np.concatenate([ye, yc])
        cen = np.concatenate([np.zeros(100, np.int32), np.ones(100, np.int32)])
        S, s = perturbed(n, 800 + n)
        out[f"n{n}_S"], out[f"n{n}_s"], out[f"n{n}_y"], out[f"n{n}_cen"] = S, s, y, cen
    for i, (n, method, mhit) in enumerate(G3_CASES):
        seed = 9000 + i
        orc.set_seed(seed)
        o = orc.ref_sweep(method, out[f"n{n}_S"], out[f"n{n}_s"], out[f"n{n}_y"], out[f"n{n}_cen"], mhit=mhit)
        B, z, N, nw = o["B"], o["z"], o["N"], o["nword"]
        k = f"n{n}_m{method}_h{mhit}"
        out[k + "_seed"] = np.int64(seed)
        out[k + "_B"] = B.astype(np.int32)
        out[k + "_z"] = z
        out[k + "_N"] = N.astype(np.int16)
        out[k + "_nw"] = nw
    return out


def _g5_case(args):
    name, seed = args
    from oracle import posterior as PO

    orc = O.OracleLib()
    n, method, mhit, y, cen, T, nu, zeta = PO.case_inputs(name)
    it = PO.CASES[name][-1]
    orc.set_seed(seed)
    chain = orc.gibbs(0, it + 1, mhit, method, n, nu, zeta, T.reshape(-1, order="F"), np.ones(T.size), y, cen)
    return name, seed, PO.summarize(chain)


def g5(orc):
    """G5 ``g5_posterior.npz``: posterior summaries (mean, 5/50/95 % quantiles,
    batch-means MCSE) of "ref"-variant chains for oracle/posterior.py CASES."""
    import multiprocessing as mp

    from oracle import posterior as PO

    del orc
    jobs = [(name, 7000 + i) for i, name in enumerate(PO.CASES)]
    with mp.get_context("fork").Pool(min(len(jobs), 7)) as pool:
        res = pool.map(_g5_case, jobs)
    out = {}
    for name, seed, summ in res:
        out.update(PO.pack(name, summ))
        out[f"{name}_seed"] = np.int64(seed)
    return out


def main():
    O.build()
    orc = O.OracleLib()
    os.makedirs(OUT, exist_ok=True)
    check = "--check" in sys.argv
    want = {a for a in sys.argv[1:] if not a.startswith("--")}
    for name, fn in (("g1_test_scripts", g1), ("g2_cfg1", g2), ("g3_sweeps", g3), ("g5_posterior", g5)):
        if want and name not in want:
            continue
        d = fn(orc)
        path = os.path.join(OUT, name + ".npz")
        if check:
            old = np.load(path)
            bad = [k for k in d if k not in old or not np.array_equal(np.asarray(d[k]), old[k])]
            bad += [k for k in old.files if k not in d]
            print(name, "identical" if not bad else f"DIFFERS in {bad}")
            continue
        np.savez_compressed(path, **d)
        print(name, os.path.getsize(path), "bytes")


if __name__ == "__main__":
    main()
