"""The R boundary without R: tests/fake_r/fake_r_host.c plays R (exports the
R API symbols, loads the library RTLD_LOCAL like dyn.load, calls
R_init_PhaseType like library(PhaseType), calls the registered routine like
.C(LJMA_Gibbs, ...)).

CPU: registration matches src/Registrations.c:6-20 (one .C routine,
15 args, INTSXP=13 / REALSXP=14 types, no dynamic symbols, forced symbols);
the library detects R; without a GPU the call ends in Rf_error (R's error
path), never in a CPU fallback.
GPU: the same call runs the reference's two test scripts as .C vectors
(tests/phtMCMC2.R, ECS, 20 iterations; tests/phtMCMC.R,
dense MHRS, m = 9, 6 iterations) on the device, with R's generator
(the host compiles phasetype_amd/csrc/rstream.c: MT19937 + R's set.seed,
unif_rand, rgamma) seeded as the scripts seed it.  The chain must equal, bit
for bit, the oracle's device-spec LJMA_Gibbs (oracle gibbs dev=1) under the
same seed: the library inside "R" draws its Philox key and every Gamma
update from R's stream exactly as the specification does.
"""
import sys
import json
import os
import subprocess

import numpy as np
import pytest

import phasetype_amd as P
from phasetype_amd import build as B

HERE = os.path.dirname(os.path.abspath(__file__))
SRC = os.path.join(HERE, "fake_r", "fake_r_host.c")
EXE = os.path.join(HERE, "fake_r", "fake_r_host")


CSRC = os.path.join(os.path.dirname(HERE), "phasetype_amd", "csrc")
DEPS = [SRC, os.path.join(HERE, "fake_r", "r_api.list"), os.path.join(CSRC, "rstream.c"),
        os.path.join(CSRC, "rstream.h")]


def _host():
    if not os.path.exists(EXE) or os.path.getmtime(EXE) < max(os.path.getmtime(d) for d in DEPS):
        # only the R API is exported: the library's own symbols stay its own
        subprocess.run(["gcc", "-O1", "-ffp-contract=off", f"-I{CSRC}",
                        f"-Wl,--dynamic-list={os.path.join(HERE, 'fake_r', 'r_api.list')}", "-o", EXE, SRC,
                        os.path.join(CSRC, "rstream.c"), "-ldl", "-lm"], check=True)
    return EXE


def _run(it, script="phtMCMC2", seed=None):
    P.load()
    env = dict(os.environ)
    path, prefix = P._lapack_path()
    env["PHT_LAPACK_LIB"], env["PHT_LAPACK_PREFIX"] = path, prefix
    argv = [_host(), B.LIB, str(it), script] + ([str(seed)] if seed is not None else [])
    r = subprocess.run(argv, capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stdout + r.stderr
    return json.loads(r.stdout.strip().splitlines()[-1])


def _no_gpu():
    try:
        return P.device_count() == 0
    except P.PhaseTypeError:
        return True


def test_registration_matches_reference():
    d = _run(3)
    assert d["routines"] == 1 and d["name"] == "LJMA_Gibbs" and d["nargs"] == 15
    assert d["types"] == [13, 13, 13, 13, 13, 14, 14, 13, 14, 14, 13, 13, 14, 13, 14]
    assert d["dynamic"] == 0 and d["force"] == 1
    assert d["in_R"] == 1


@pytest.mark.skipif(not _no_gpu(), reason="a HIP device is present")
def test_no_gpu_raises_r_error():
    d = _run(3)
    assert d["errored"] == 1 and "HIP" in d["error"]
    assert d["getrng"] == d["putrng"] == 1  # RNG state saved back to R before the error


def _script_args(script):
    sys.path.insert(0, os.path.join(os.path.dirname(HERE), "tools"))
    import make_golden as G

    return G.X20, (G.PHTMCMC2_ARGS if script == "phtMCMC2" else G.PHTMCMC_ARGS)


@pytest.mark.gpu
@pytest.mark.parametrize("script", ["phtMCMC2", "phtMCMC"])
def test_reference_test_scripts_through_fake_r(orc, script):
    """tests/phtMCMC2.R and tests/phtMCMC.R (R/phtMCMC2.R:73, R/phtMCMC.R:83)
    through R_init_PhaseType -> the registered LJMA_Gibbs on the GPU, with
    R's stream: bit-equal to the oracle's device-spec LJMA_Gibbs."""
    x, a = _script_args(script)
    it, m = a["it"], len(a["nu"])
    d = _run(it, script)
    assert d["errored"] == 0, d["error"]
    assert d["finite"] == 1 and d["m"] == m
    got = np_res(d, it, m)
    orc.set_seed(a["seed"])
    want = orc.gibbs(1, it, a["mhit"], a["method"], a["n"], a["nu"], a["zeta"], np.array(a["T"], np.int32),
                     np.ones(16), x, np.zeros(20, np.int32))
    assert np.array_equal(got, want), (got[:3], want[:3])
    nu, zeta = np.array(a["nu"]), np.array(a["zeta"])
    mode = nu > 1
    assert np.array_equal(got[0][mode], ((nu - 1) / zeta)[mode])  # row 0: the prior mode (nu > 1)
    # R's stream: one rgamma per parameter per sweep, plus one per nu <= 1 at the start
    assert d["gamma"] == m * (it - 1) + int((~mode).sum())
    assert d["getrng"] == d["putrng"] == 1


@pytest.mark.gpu
def test_fake_r_seed_changes_the_chain():
    a = _run(8, "phtMCMC2", seed=1)
    b = _run(8, "phtMCMC2", seed=2)
    assert a["errored"] == 0 and b["errored"] == 0
    assert a["res"] != b["res"]


def np_res(d, it, m):
    """res (column-major it x m, res[iter + i*it]) as [it, m]."""
    return np.array(d["res"]).reshape(m, it).T
