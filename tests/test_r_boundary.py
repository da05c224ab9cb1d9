"""The R boundary without R: tests/fake_r/fake_r_host.c plays R (exports the
R API symbols, loads the library RTLD_LOCAL like dyn.load, calls
R_init_PhaseType like library(PhaseType), calls the registered routine like
.C(LJMA_Gibbs, ...)).

CPU: registration matches src/Registrations.c:6-20 (one .C routine,
15 args, INTSXP=13 / REALSXP=14 types, no dynamic symbols, forced symbols);
the library detects R; without a GPU the call ends in Rf_error (R's error
path), never in a CPU fallback.
GPU: the same call runs the tests/phtMCMC2.R chain on the device with R's
(stand-in) RNG: row 0 is the prior mean, every draw finite and positive.
"""
import json
import os
import subprocess

import pytest

import phasetype_amd as P
from phasetype_amd import build as B

HERE = os.path.dirname(os.path.abspath(__file__))
SRC = os.path.join(HERE, "fake_r", "fake_r_host.c")
EXE = os.path.join(HERE, "fake_r", "fake_r_host")


def _host():
    if not os.path.exists(EXE) or os.path.getmtime(EXE) < os.path.getmtime(SRC):
        subprocess.run(["gcc", "-O1", "-rdynamic", "-o", EXE, SRC, "-ldl", "-lm"], check=True)
    return EXE


def _run(it):
    P.load()
    env = dict(os.environ)
    path, prefix = P._lapack_path()
    env["PHT_LAPACK_LIB"], env["PHT_LAPACK_PREFIX"] = path, prefix
    r = subprocess.run([_host(), B.LIB, str(it)], capture_output=True, text=True, timeout=300, env=env)
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


@pytest.mark.gpu
def test_chain_through_fake_r():
    it = 20
    d = _run(it)
    assert d["errored"] == 0, d["error"]
    assert d["finite"] == 1
    assert d["row0"] == [1.4375, 11.1875]  # prior mean nu/zeta
    assert d["gamma"] == 2 * (it - 1)  # one rgamma per parameter per sweep, from R's stream
    assert d["getrng"] == d["putrng"] == 1
