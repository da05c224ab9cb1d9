"""oracle/cpu_best.py — TEST INFRASTRUCTURE ONLY (bench.py's CPU comparison).

The "best CPU" line of SURVEY.md §8(d): the CPU restatement of the reference
(oracle/, "ref" variant, LJMA_Gibbs as R's .C calls it) on W host cores at
once, the observations split W ways.  The reference is single-threaded and
its per-sweep work is linear in the observations, so W processes each running
the restatement over 1/W of a bounded sample measure what an ideal
observation-parallel CPU port would reach: value = W x (sweeps/s over
N_sample / W) x N_sample / N, with the wall time of the slowest worker.  The
per-sweep reduction such a port needs is not charged (it favours the CPU).

Run as a child process (bench.py does: the GPU process never forks workers):
    python3 -m oracle.cpu_best --n 10 --N 1000000 --workers 16 --seconds 10
Prints one JSON object.  (The reference itself needs R and cannot be built in
this image)
"""
from __future__ import annotations

import argparse
import json
import multiprocessing as mp
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))

from phasetype_amd.synth import DATA_KEY, bd_exit, bd_exit_structure, simulate_ph  # noqa: E402


def _runner(n, method=2):
    from oracle import oracle as O

    T, theta = bd_exit_structure(n)
    nu, zeta = 1.0 + 50.0 * theta, np.full(len(theta), 50.0)
    Tf = T.reshape(-1, order="F")
    lib = O.OracleLib()
    return "port", lambda it, y, c: lib.gibbs(0, it, 1, method, n, nu, zeta, Tf, np.ones(T.size), y, c), lib


def _worker(args):
    n, method, y, c, sweeps, t_start = args
    _, run, lib = _runner(n, method)
    lib.set_seed(3)
    while time.time() < t_start:  # common start, so the slowest worker's wall is the job's
        time.sleep(0.001)
    t0 = time.perf_counter()
    run(sweeps + 1, y, c)
    return time.perf_counter() - t0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=10)
    ap.add_argument("--N", type=int, default=1_000_000)
    ap.add_argument("--censor", type=float, default=0.0)
    ap.add_argument("--workers", type=int, default=16)
    ap.add_argument("--seconds", type=float, default=10.0)
    ap.add_argument("--method", type=int, default=2)
    a = ap.parse_args()
    S, s = bd_exit(a.n)
    y, cen = simulate_ph(S, s, a.N, seed=DATA_KEY, censor_frac=a.censor)
    W = max(1, min(a.workers, os.cpu_count() or 1))
    kind, run, lib = _runner(a.n, a.method)
    lib.set_seed(1)
    probe = min(len(y), 20000)
    t0 = time.perf_counter()
    run(2, y[:probe], cen[:probe])
    per_obs_sweep = (time.perf_counter() - t0) / max(probe, 1)
    # each worker: ~`seconds` of work over its share of the sample
    per_w = int(min(len(y) // W, max(2000, a.seconds / max(per_obs_sweep * 5, 1e-12))))
    sweeps = max(2, min(50, int(a.seconds / max(per_obs_sweep * per_w, 1e-12))))
    nsamp = per_w * W
    jobs = [(a.n, a.method, np.ascontiguousarray(y[k * per_w:(k + 1) * per_w]), np.ascontiguousarray(cen[k * per_w:(k + 1) * per_w]),
             sweeps, time.time() + 1.0) for k in range(W)]
    with mp.get_context("fork").Pool(W) as pool:
        walls = pool.map(_worker, jobs)
    wall = max(walls)
    value = (sweeps / wall) * nsamp / len(y)
    print(json.dumps({"value": value, "unit": "iterations/s", "cores": W, "kind": kind,
                      "sample": f"{sweeps} Gibbs sweeps over {nsamp} of the {len(y)} observations split over {W} "
                                f"processes ({per_w} each; slowest {wall:.1f} s, fastest {min(walls):.1f} s), "
                                f"scaled by {nsamp}/{len(y)} to N={len(y)}; ideal observation-parallel CPU, "
                                f"per-sweep reduction not charged"}))


if __name__ == "__main__":
    main()
