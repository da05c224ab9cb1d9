#!/usr/bin/env python3
"""Kernel time of the ECS-exact sweep against the shard size (strong-scaling
regime) for the launch variants the host can pick at run time:
PHT_GROUP (lanes per observation), PHT_ECS_OCC (blocks per CU), PHT_HOT
(variant hotK: wave priority for the K longest remaining paths), PHT_ROWK (variant rowK:
the K longest observations on 16-lane rows), base = defaults.

usage (GPU box): python3 tools/latency.py [--Ns 62500 125000 ...] [--sweeps 8]
       python3 tools/latency.py --shards 8 [--sweeps 8]
Shard = the first N observations of the bench data set (what rank 0 of
1e6/N GPUs holds).  "topK" entries use the K largest observations instead
(one lone wavefront for K=64: the per-round latency of the longest paths).
Every variant must reproduce the first variant's draws (identical results).
Prints one JSON object per shard size.

--shards W: the real W-GPU partition: every shard
shard_range(1e6, r, W), r = 0..W-1, with its global ids (obs0 = lo, the
Philox counters an 8-GPU run uses), swept on this one GPU in turn.  The
W-GPU sweep is the maximum over them (plus RCCL's latency), so the line
reports per shard the kernel and sweep ms (median over --sweeps Gibbs
sweeps) and which shard holds the global longest observation, then the
max, median and the projected speed-up over the whole set on one GPU.
"""
import argparse
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import phasetype_amd as P  # noqa: E402
from phasetype_amd.synth import DATA_KEY, bd_exit, bd_exit_structure, simulate_ph  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=10)
    ap.add_argument("--Ns", nargs="+", default=["top4096", "31250", "62500", "125000", "250000", "500000", "1000000"])
    ap.add_argument("--variants", nargs="+", default=["g1o2", "sp", "g4"])
    ap.add_argument("--sweeps", type=int, default=8)
    ap.add_argument("--shards", type=int, default=0)
    ap.add_argument("--N", type=int, default=1_000_000)
    ap.add_argument("--data", type=int, default=1_000_000, help="size of the bench data set the Ns specs index")
    a = ap.parse_args()
    if a.shards:
        return shards(a)
    n = a.n
    S, s = bd_exit(n)
    T, theta = bd_exit_structure(n)
    nu, zeta = 1 + 50 * theta, np.full(len(theta), 50.0)
    y, cen = simulate_ph(S, s, a.data, seed=DATA_KEY, censor_frac=0.0)
    zexp = P.zexp_for(y)
    Cm = np.ones(T.shape)
    for spec in a.Ns:
        if spec.startswith("rand"):
            k = int(spec[4:])
            idx = np.sort(np.random.default_rng(11).choice(len(y), k, replace=False))
        elif spec.startswith("drop"):  # dropKofS: the first S observations without their K largest
            k, sz = (int(v) for v in spec[4:].split("of"))
            first = np.arange(sz)
            idx = np.sort(first[np.argsort(-y[:sz])[k:]])
        elif spec.startswith("top"):
            k = int(spec[3:])
            idx = np.sort(np.argsort(-y)[:k])
        else:
            idx = np.arange(int(spec))
        ys, cs = np.ascontiguousarray(y[idx]), np.ascontiguousarray(cen[idx])
        sw = P.Sweeper(n, 2, 1, device=0)
        sw.set_obs(ys, cs, obs0=0)
        out = {"N": spec}
        ref = None
        for v in a.variants:
            os.environ.pop("PHT_GROUP", None)
            os.environ.pop("PHT_ECS_OCC", None)
            os.environ.pop("PHT_SPREAD", None)
            os.environ.pop("PHT_NEWCAP", None)
            os.environ.pop("PHT_HOT", None)
            os.environ.pop("PHT_ROWK", None)
            os.environ.pop("PHT_ROWPRIO", None)
            if v == "base":
                pass
            elif v.startswith("row"):  # rowK[pP]: the K longest observations on 16-lane rows (wave priority P)
                k, _, pr = v[3:].partition("p")
                os.environ["PHT_ROWK"] = k
                if pr:
                    os.environ["PHT_ROWPRIO"] = pr
            elif v.startswith("hot"):  # waves with one of the K longest remaining paths at high priority
                os.environ["PHT_HOT"] = v[3:]
            elif v.startswith("nc"):
                os.environ["PHT_GROUP"] = "1"
                os.environ["PHT_NEWCAP"] = v[2:]
            elif v == "sp":
                os.environ["PHT_GROUP"] = "1"
                os.environ["PHT_SPREAD"] = "1"
            elif v.startswith("g1o"):
                os.environ["PHT_GROUP"] = "1"
                os.environ["PHT_ECS_OCC"] = v[3:]
            else:
                os.environ["PHT_GROUP"] = v[1:]
            P.set_seed(5)
            sw.gibbs(2, 2, nu, zeta, T, Cm, zexp)  # warm-up
            P.set_seed(7)
            sw.kernel_ms_total = 0.0
            t0 = time.perf_counter()
            res = sw.gibbs(a.sweeps + 1, 2, nu, zeta, T, Cm, zexp)
            dt = time.perf_counter() - t0
            same = True
            if ref is None:
                ref = res
            else:
                same = bool(np.array_equal(ref, res))
            out[v] = {"kernel_ms": round(sw.kernel_ms_total / a.sweeps, 4),
                      "sweep_ms": round(dt / a.sweeps * 1e3, 4), "same": same}
        sw.close()
        print(json.dumps(out), flush=True)


def shards(a):
    from phasetype_amd.dist import shard_range

    n, W = a.n, a.shards
    S, s = bd_exit(n)
    T, theta = bd_exit_structure(n)
    nu, zeta = 1 + 50 * theta, np.full(len(theta), 50.0)
    y, cen = simulate_ph(S, s, a.N, seed=DATA_KEY, censor_frac=0.0)
    zexp = P.zexp_for(y)  # every rank uses the global exponent
    Cm = np.ones(T.shape)
    top = int(np.argmax(y))

    def run(lo, hi):
        sw = P.Sweeper(n, 2, 1, device=0)
        sw.set_obs(y[lo:hi], cen[lo:hi], obs0=lo)
        P.set_seed(5)
        w = sw.gibbs(3, 2, nu, zeta, T, Cm, zexp)  # warm-up
        ks, ts = [], []
        for rep in range(3):  # median of 3 timed runs of --sweeps sweeps each
            P.set_seed(100 + rep)
            t0 = time.perf_counter()
            sw.gibbs(a.sweeps + 1, 2, nu, zeta, T, Cm, zexp, start=w[-1])
            ts.append((time.perf_counter() - t0) * 1e3 / a.sweeps)
            ks.append(sw.kernel_ms_total / a.sweeps)
        sw.close()
        return float(np.median(ks)), float(np.median(ts))

    k1, t1 = run(0, a.N)
    rows = []
    for r in range(W):
        lo, hi = shard_range(a.N, r, W)
        k, t = run(lo, hi)
        rows.append({"rank": r, "lo": lo, "hi": hi, "kernel_ms": round(k, 4), "sweep_ms": round(t, 4),
                     "holds_longest": bool(lo <= top < hi), "ymax": round(float(y[lo:hi].max()), 3)})
        print(json.dumps(rows[-1]), flush=True)
    km = max(r["kernel_ms"] for r in rows)
    tm = max(r["sweep_ms"] for r in rows)
    print(json.dumps({"shards": W, "N": a.N, "n": n, "one_gpu_kernel_ms": round(k1, 4),
                      "one_gpu_sweep_ms": round(t1, 4), "max_kernel_ms": km,
                      "median_kernel_ms": float(np.median([r["kernel_ms"] for r in rows])),
                      "max_sweep_ms": tm, "longest_on_rank": [r["rank"] for r in rows if r["holds_longest"]],
                      "global_ymax": round(float(y[top]), 3),
                      "projected_speedup_sweep": round(t1 / tm, 3),
                      "note": "sweep ms includes the host per-sweep work; an 8-GPU run adds RCCL's all-reduce"}),
          flush=True)


if __name__ == "__main__":
    main()
