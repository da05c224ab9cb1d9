#!/usr/bin/env python3
"""Interleaved A/B timing of libPhaseType.so variants, one persistent worker
process per variant (cdna_hip_programming.md §5.4 rule 24: interleaved
rounds on one box).

Why not one process: a second library's context in the same process gets
its two streams mapped onto hardware queues that serialise them, so the ECS
censored range no longer overlaps the exact range (r03: n = 15, 30 %
censored, 1.46 ms alone vs 2.44 ms as the second library; profiles/r03/
ab_isolation/).  Each worker owns one library; the parent sends "run" in
interleaved order and only one worker uses the GPU at a time.

usage (GPU box): python3 tools/ab.py --libs a.so b.so ... [--rounds 5 --sweeps 10]
A library may carry environment settings for its worker: "a.so@PHT_ECS_OCC=1,PHT_ROWK=0"
(the same library twice with different knobs is two variants).
Each variant runs the bench workload (BD-exit(n), N obs, ECS) as a Gibbs
run of --sweeps sweeps per round; rounds interleave the variants.  Prints a
JSON summary: per-variant median / min ms per sweep and kernel ms.
Every variant must also reproduce variant 0's Gibbs draws exactly (same
seed) — the A/B is only meaningful between bit-identical variants.
"""
import argparse
import ctypes as C
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import phasetype_amd as P  # noqa: E402
from phasetype_amd.synth import DATA_KEY, bd_exit, bd_exit_structure, simulate_ph  # noqa: E402

_dp = np.ctypeslib.ndpointer(dtype=np.float64, flags="C_CONTIGUOUS")
_ip = np.ctypeslib.ndpointer(dtype=np.int32, flags="C_CONTIGUOUS")


class Lib:
    def __init__(self, path, n, method, y, cen):
        self.L = L = C.CDLL(os.path.abspath(path), mode=C.RTLD_LOCAL)
        L.pht_last_error.restype = C.c_char_p
        L.pht_bind_lapack.argtypes = [C.c_char_p, C.c_char_p]
        L.pht_set_seed.argtypes = [C.c_uint32]
        L.pht_ctx_create.restype = C.c_void_p
        L.pht_ctx_create.argtypes = [C.c_int, C.c_int, C.c_int, C.c_int]
        L.pht_ctx_set_obs.argtypes = [C.c_void_p, _dp, _ip, C.c_long, C.c_long]
        L.pht_gibbs_run.argtypes = [C.c_void_p, C.c_int, C.c_int, C.c_int, _dp, _dp, _ip, _dp, C.c_int, C.c_int,
                                    _dp, _dp, C.c_void_p, C.c_void_p, C.POINTER(C.c_double)]
        p, pre = P._lapack_path()
        assert L.pht_bind_lapack(p.encode(), pre.encode()) == 0
        self.ctx = L.pht_ctx_create(0, n, method, 1)
        assert self.ctx, L.pht_last_error()
        assert L.pht_ctx_set_obs(self.ctx, y, cen, len(y), 0) == 0

    def run(self, it, method, nu, zeta, T, Cm, zexp, seed):
        m = len(nu)
        res = np.zeros(it * m)
        kms = C.c_double()
        self.L.pht_set_seed(seed)
        t0 = time.perf_counter()
        rc = self.L.pht_gibbs_run(self.ctx, it, method, m, nu, zeta, T, Cm, zexp, 1, np.array([-1.0]), res, None,
                                  None, C.byref(kms))
        dt = time.perf_counter() - t0
        assert rc == 0, self.L.pht_last_error()
        return dt, kms.value, res


def _split(spec):
    path, _, env = spec.partition("@")
    return path, dict(kv.split("=", 1) for kv in env.split(",") if kv)


def _worker(conn, spec, n, method, y, cen):
    path, env = _split(spec)
    os.environ.update(env)
    lb = Lib(path, n, method, y, cen)
    while True:
        msg = conn.recv()
        if msg is None:
            break
        conn.send(lb.run(*msg))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--libs", nargs="+", required=True)
    ap.add_argument("--n", type=int, default=10)
    ap.add_argument("--N", type=int, default=1_000_000)
    ap.add_argument("--method", default="ECS")
    ap.add_argument("--censor", type=float, default=0.0)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--sweeps", type=int, default=10)
    ap.add_argument("--no-check", action="store_true", help="timing-only variants (results differ)")
    a = ap.parse_args()
    n = a.n
    method = P.METHODS[a.method]
    S, s = bd_exit(n)
    T, theta = bd_exit_structure(n)
    nu, zeta = 1 + 50 * theta, np.full(len(theta), 50.0)
    y, cen = simulate_ph(S, s, a.N, seed=DATA_KEY, censor_frac=a.censor)
    zexp = P.zexp_for(y)
    Tf = np.ascontiguousarray(T.reshape(-1, order="F"), np.int32)
    Cm = np.ones(T.size)
    import multiprocessing as mp
    ctx = mp.get_context("spawn")
    libs, procs = [], []
    for p in a.libs:
        pc, cc = ctx.Pipe()
        pr = ctx.Process(target=_worker, args=(cc, p, n, method, y, cen), daemon=True)
        pr.start()
        libs.append(pc)
        procs.append(pr)

    def run(conn, *args):
        conn.send(args)
        return conn.recv()

    for lb in libs:  # warm-up
        run(lb, 3, method, nu, zeta, Tf, Cm, zexp, 1)
    times = {p: [] for p in a.libs}
    kern = {p: [] for p in a.libs}
    ref = None
    for r in range(a.rounds):
        for p, lb in zip(a.libs, libs):
            dt, kms, res = run(lb, a.sweeps + 1, method, nu, zeta, Tf, Cm, zexp, 100 + r)
            if r == 0 and not a.no_check:
                if ref is None:
                    ref = res
                elif not np.array_equal(ref, res):
                    print(json.dumps({"error": f"{p} draws differ from {a.libs[0]}"}))
            times[p].append(dt / a.sweeps * 1e3)
            kern[p].append(kms / a.sweeps)
    out = {(os.path.basename(_split(p)[0]) + ("@" + p.partition("@")[2] if "@" in p else "")): {"ms_per_sweep_median": float(np.median(times[p])), "ms_min": float(np.min(times[p])),
                                 "kernel_ms_median": float(np.median(kern[p]))} for p in a.libs}
    print(json.dumps(out, indent=1))
    for lb, pr in zip(libs, procs):
        lb.send(None)
        pr.join(60)


if __name__ == "__main__":
    main()
