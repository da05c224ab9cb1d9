"""Build the native library in-tree: phasetype_amd/_lib/libPhaseType.so.

hipcc for gfx950: the HIP kernels (pht_kernels_nt.hip once per compile-time
n, in parallel, + the pht_dispatch.hip launcher), the host runtime / C ABI
(gibbs_host.cpp) and the R-compatible stream (rstream.c), then one link.
``-ffp-contract=off`` is required: the device path must reproduce the
oracle's arithmetic bit for bit (no implicit FMA contraction anywhere).
"""
from __future__ import annotations

import os
import shutil
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
CSRC = os.path.join(HERE, "csrc")
OUT_DIR = os.path.join(HERE, "_lib")
LIB = os.path.join(OUT_DIR, "libPhaseType.so")
KERNEL_NTS = (10, 3, 5, 15, 20, 0)  # compile-time n of the kernels (0 = runtime n)
# the n = 10 unit (the headline kernel) with the machine scheduler weighting
# latency over occupancy: the same occupancy for every kernel of the unit
# (tests/test_kernel_regs.py), ECS cfg4 kernel -0.7 / -0.8 % in two
# interleaved A/Bs on two boxes (profiles/r05/sched_flags/); not for n = 15,
# where cfg5 ECS lost 0.9 / 2.4 %
UNIT_FLAGS = {10: ("-mllvm", "--amdgpu-schedule-metric-bias=0")}
# Philox blocks with their ten rounds unrolled (the compiler keeps a loop of
# two rounds otherwise; the same words): every kernel of the n = 5 and n = 20
# units (cfg2 -4.1 %, cfg3 -1.4 % per sweep), the MHRS search of the n = 15
# unit (cfg5 MHRS -1.4 %; every n = 15 kernel unrolled lost 3.9 % at cfg5 ECS)
# and the ECS exact kernel's top-up at n = 10 and 15 (cfg4 -0.7 %, cfg5 ECS
# -0.9 %; the censored kernel's: neutral) (profiles/r06/unroll/)
UNIT_DEFINES = {5: ("PHT_PHILOX_UNROLL",), 20: ("PHT_PHILOX_UNROLL",),
                10: ("PHT_ECS_PHILOX_UNROLL",), 15: ("PHT_MHRS_PHILOX_UNROLL", "PHT_ECS_PHILOX_UNROLL")}
# (source, extra defines, extra device-compile flags) per object
UNITS = [("pht_kernels_nt.hip", (f"PHT_NT={k}",) + UNIT_DEFINES.get(k, ()), UNIT_FLAGS.get(k, ()))
         for k in KERNEL_NTS] + [
    ("pht_dispatch.hip", (), ()), ("pht_resident.hip", (), ()), ("gibbs_host.cpp", (), ()), ("rstream.c", (), ())]
SOURCES = sorted({u[0] for u in UNITS})
HEADERS = ["pht_device.h", "pht_env.h", "pht_kernels.h", "pht_kernels_impl.h", "pht_layout.h", "rstream.h",
           "pht_ecs_round.h", "pht_ecs_row.h", "pht_dcs_round.h", "pht_cens_round.h", "pht_unif.h"]
ARCH = os.environ.get("PYTORCH_ROCM_ARCH", "gfx950").split(";")[0]
DEFAULT_DEFINES: tuple = ("PHT_DETMATH_LDS",)


def _hipcc() -> str:
    for c in (shutil.which("hipcc"), "/opt/rocm/bin/hipcc"):
        if c and os.path.exists(c):
            return c
    raise RuntimeError("hipcc not found")


def inputs() -> list:
    """Every file the default library is built from (sources, headers, this
    script with its flags)."""
    deps = [os.path.join(CSRC, f) for f in SOURCES + HEADERS]
    deps += [os.path.join(REPO, "include", f) for f in ("phasetype_amd.h", "pht_detmath.h", "pht_philox.h",
                                                          "pht_gamma.h", "pht_eigen.h")]
    deps.append(os.path.abspath(__file__))
    return deps


def source_key() -> str:
    """sha256 over the default library's build inputs (name + content): the
    same for every build of the same sources, wherever it was compiled (the
    .so itself embeds its build directory)."""
    import hashlib

    h = hashlib.sha256()
    for d in inputs():
        h.update(os.path.relpath(d, REPO).encode() + b"\0")
        with open(d, "rb") as f:
            h.update(f.read())
    return h.hexdigest()


def needs_build() -> bool:
    if not os.path.exists(LIB):
        return True
    t = os.path.getmtime(LIB)
    return any(os.path.getmtime(d) > t for d in inputs() if os.path.exists(d))


def _merge_defines(defines) -> list:
    """DEFAULT_DEFINES, with any macro that ``defines`` names replaced."""
    names = {d.split("=")[0] for d in defines}
    return [d for d in DEFAULT_DEFINES if d.split("=")[0] not in names] + list(defines)


def build(force: bool = False, verbose: bool = False, defines=(), out: str | None = None, flags=()) -> str:
    """Compile; ``defines`` (e.g. ["PHT_DETMATH_LDS"]), extra device-compile
    ``flags`` and ``out`` build a variant library elsewhere (tools/ab.py)
    without touching the default."""
    target = out or LIB
    if not force and not defines and not flags and out is None and not needs_build():
        return LIB
    os.makedirs(OUT_DIR, exist_ok=True)

    def compile_unit(idx_unit):
        idx, (src, extra, uflags) = idx_unit
        path = os.path.join(CSRC, src)
        obj = os.path.join(OUT_DIR, f"{os.path.basename(target)}.{idx}.{src}.o")
        cmd = [_hipcc(), "-O3", "-fPIC", "-ffp-contract=off", f"-I{os.path.join(REPO, 'include')}", f"-I{CSRC}",
               "-Wno-pass-failed"] + [f"-D{d}" for d in _merge_defines(tuple(defines) + tuple(extra))]
        if src.endswith(".hip"):
            cmd += ["-x", "hip", f"--offload-arch={ARCH}", "-std=c++17"] + list(uflags) + list(flags)
        elif src.endswith(".cpp"):
            cmd += ["-x", "c++", "-std=c++17", "-D__HIP_PLATFORM_AMD__", "-I/opt/rocm/include"]
        else:
            cmd += ["-x", "c", "-std=gnu11"]
        cmd += ["-c", path, "-o", obj]
        if verbose:
            print(" ".join(cmd), file=sys.stderr)
        subprocess.run(cmd, check=True)
        return obj

    workers = max(1, min(len(UNITS), int(os.environ.get("MAX_JOBS", os.cpu_count() or 4)), 8))
    with ThreadPoolExecutor(max_workers=workers) as ex:
        objs = list(ex.map(compile_unit, enumerate(UNITS)))
    tmp = target + ".tmp"
    cmd = [_hipcc(), "-shared", "-fPIC", f"--offload-arch={ARCH}", "-o", tmp] + objs + ["-ldl"]
    subprocess.run(cmd, check=True)
    os.replace(tmp, target)
    for o in objs:
        os.remove(o)
    return target


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True))
