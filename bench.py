#!/usr/bin/env python3
"""bench.py — Gibbs iterations/s of the PhaseType hot path on MI355X.

Workload (BASELINE.json metric, configs[3] "cfg4"): phtMCMC2's default ECS
sampler on the BD-exit(n=10) generator (m = 28 parameters), N = 1e6 exact
synthetic absorption times; one *step* = one full Gibbs sweep = host
per-sweep spectral setup (P/Pfull, dgeevx, Q^-1 v, packed parameters) +
step-1 latent-path sampling of every observation on the GPU(s) + the
sufficient-statistics reduction + the host conjugate Gamma update
(src/PHT_MCMC_Aslett.c:268-405).  Nothing is skipped inside the timed
region; observations are resident in HBM before timing starts.

Multi-GPU (strong scaling, N fixed): one process per GPU, rank r owns a
contiguous shard of the observations; each sweep's int64 statistics block is
summed across ranks with one all-reduce (torch.distributed, backend "nccl" =
RCCL over xGMI) and every rank draws the identical Gamma update.

Prints ONE JSON line on rank 0 (see DESIGN.md §Measurement for the
roofline and cpu_baseline fields).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

import phasetype_amd as P  # noqa: E402
from phasetype_amd.dist import attach_rccl, make_stats_allreduce, max_over_ranks, shard_range, sum_over_ranks  # noqa: E402
from phasetype_amd.synth import DATA_KEY, bd_exit, bd_exit_structure, simulate_ph  # noqa: E402

HBM_PEAK_GBS = 8000.0     # MI355X HBM3E peak (MI355X_MICROARCH.md, spec)
FP64_VALU_PEAK_TF = 78.6  # MI355X FP64 vector peak (spec)
ALG_BYTES_PER_OBS = 12    # y f64 + censored i32 per observation per sweep


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def cpu_baseline(n, y, cen, T, nu, zeta, method=2, target_s=15.0):
    """The CPU restatement of the reference (oracle/, "ref" variant: R's
    stream, libm, the reference's arithmetic order; kind "port") timed
    single-threaded on a bounded sample of the same workload.  The reference
    itself needs R and cannot be built in this image."""
    from oracle import oracle as O

    kind = "port"
    lib = O.OracleLib()
    run = lambda it, yy, cc: lib.gibbs(0, it, 1, method, n, nu, zeta, T.reshape(-1, order="F"),  # noqa: E731
                                       np.ones(T.size), yy, cc)
    lib.set_seed(1)
    probe = 20000
    t0 = time.perf_counter()
    run(2, y[:probe], cen[:probe])
    per_obs_sweep = (time.perf_counter() - t0) / probe
    nsamp = int(min(len(y), max(20000, 200000)))
    sweeps = max(2, int(target_s / max(per_obs_sweep * nsamp, 1e-9)))
    sweeps = min(sweeps, 50)
    lib.set_seed(2)
    t0 = time.perf_counter()
    run(sweeps + 1, y[:nsamp], cen[:nsamp])
    dt = time.perf_counter() - t0
    rate_sample = sweeps / dt
    value = rate_sample * nsamp / len(y)  # sweeps/s scaled to the full N (work is linear in N)
    return {"value": value, "unit": "iterations/s", "cores": 1, "kind": kind,
            "sample": f"{sweeps} Gibbs sweeps over the first {nsamp} of the {len(y)} observations "
                      f"({dt:.1f} s, {rate_sample:.4f} sweeps/s), scaled by {nsamp}/{len(y)} to N={len(y)}; "
                      f"single thread of the GPU box's host CPU"}


def load_counters(path, n, n_local, method, lib_key):
    """PMC counters of profiles/traffic_latest.json for this workload, or
    (None, None, reason).  Fail closed: the file must name the sha256 of the
    library this process loaded (the counters were measured on that build)
    and the same (n, local N, method); otherwise the line carries no
    traffic and no FP64-VALU roofline."""
    if not os.path.exists(path):
        return None, None, "no counter file"
    try:
        tf = json.load(open(path))
    except Exception as e:  # noqa: BLE001
        return None, None, f"unreadable counter file: {e}"
    if tf.get("lib_key") != lib_key:
        return None, None, (f"counters measured on library {str(tf.get('lib_key'))[:16]}, "
                            f"this run loaded {lib_key[:16]}: not reported")
    if (tf.get("n"), tf.get("N_local"), tf.get("method")) != (n, n_local, method):
        return None, None, "counters measured on another workload"
    return tf.get("hbm_bytes_per_launch"), tf.get("fp64_flops_per_launch"), f"PMC of this library: {tf.get('pmc_dir')}"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--n", "--states", dest="n", type=int, default=10)
    ap.add_argument("--N", "--obs", dest="N", type=int, default=1_000_000)
    ap.add_argument("--method", default="ECS", choices=["ECS", "MHRS", "DCS", "UNIF"])
    ap.add_argument("--censor", type=float, default=0.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-weak", action="store_true", help="skip the weak-scaling side measurement (N > 1)")
    ap.add_argument("--no-alt", action="store_true", help="skip the UNIF side measurement")
    ap.add_argument("--traffic-file", default=os.path.join(REPO, "profiles", "traffic_latest.json"))
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    # backend "nccl" = RCCL over xGMI (one GPU per rank).  PHT_DIST_BACKEND=gloo
    # rehearses the multi-rank flow on a box with fewer GPUs than ranks (ranks
    # share devices round-robin, the statistics travel through host memory).
    backend = os.environ.get("PHT_DIST_BACKEND", "nccl")
    coll_dev = "cpu"
    # Under torchrun (WORLD_SIZE set) the process group is initialised even at
    # world 1, so `--nproc-per-node 1` runs the same RCCL code as N > 1.
    # torch initialises the device BEFORE the library loads: the library then
    # shares torch's HIP runtime (loaded the other way round, two runtimes are
    # mapped and torch's sees no device).
    if "WORLD_SIZE" in os.environ:
        import torch
        import torch.distributed as dist

        if backend == "nccl":
            torch.cuda.set_device(local)
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
            coll_dev = f"cuda:{local}"
        else:
            dist.init_process_group(backend)
            local = local % max(1, P.device_count())

    n, N = args.n, args.N
    method = P.METHODS[args.method]
    S, s = bd_exit(n)
    T, theta = bd_exit_structure(n)
    m = len(theta)
    nu, zeta = 1.0 + 50.0 * theta, np.full(m, 50.0)
    y, cen = simulate_ph(S, s, N, seed=DATA_KEY, censor_frac=args.censor)
    zexp = P.zexp_for(y)
    lo, hi = shard_range(N, rank, world)
    sw = P.Sweeper(n, method, 1, device=local)
    sw.set_obs(y[lo:hi], cen[lo:hi], obs0=lo)
    sw.set_global_count(N)  # every sweep checks that all N observations were sampled
    Cm = np.ones(T.shape)

    # On the GPUs the statistics block is summed by an RCCL all-reduce inside
    # the library, on the sweep's stream (attach_rccl); PHT_STATS_REDUCE=
    # callback (and gloo) use the host callback through torch.distributed.
    # attach_rccl self-tests the library's all-reduce against torch.distributed
    # on every rank; if that fails the run falls back to the host callback.
    in_lib = dist is not None and coll_dev != "cpu" and os.environ.get("PHT_STATS_REDUCE", "rccl") == "rccl"
    reduce = None
    reduce_note = "none"
    # one rank has nothing to sum: under torchrun at world 1 the sweep runs
    # without a collective (an RCCL all-reduce over one rank still costs
    # ~50 us per sweep, profiles/r06/torchrun/); PHT_WORLD1_REDUCE=1 keeps it
    use_coll = dist is not None and (world > 1 or os.environ.get("PHT_WORLD1_REDUCE", "0") == "1")
    if not use_coll:
        in_lib = False
        if dist is not None:
            reduce_note = "none (world 1)"
    else:
        if in_lib and not attach_rccl(sw, dist, coll_dev):
            log("[bench] in-library RCCL all-reduce failed its self-test; using the host callback")
            in_lib = False
            sw.close()
            sw = P.Sweeper(n, method, 1, device=local)
            sw.set_obs(y[lo:hi], cen[lo:hi], obs0=lo)
            sw.set_global_count(N)
            reduce_note = "host-callback (rccl self-test failed)"
        if in_lib:
            reduce_note = "rccl-in-stream (self-tested)"
        else:
            reduce = make_stats_allreduce(dist, P.stats_len(n), device=coll_dev)
            if reduce_note == "none":
                reduce_note = "host-callback"

    def sync():
        if dist is not None:
            import torch

            dist.barrier()
            if coll_dev != "cpu":
                torch.cuda.synchronize()

    P.set_seed(20241008)
    warm = sw.gibbs(args.warmup + 1, method, nu, zeta, T, Cm, zexp, reduce=reduce)
    start = warm[-1]
    sync()
    t0 = time.perf_counter()
    res = sw.gibbs(args.steps + 1, method, nu, zeta, T, Cm, zexp, start=start, reduce=reduce)
    sync()
    dt = time.perf_counter() - t0
    kernel_ms = sw.kernel_ms_total / args.steps
    if dist is not None:
        dt, kernel_ms = max_over_ranks(dist, [dt, kernel_ms], device=coll_dev)
    if not np.all(np.isfinite(res)):
        raise SystemExit("non-finite Gibbs draws")
    sw.close()

    # Side measurement (not `value`): the same workload through the opt-in
    # uniformisation sampler (method 8, pht_unif.h), which samples the same
    # conditional path law as ECS exactly and is posterior-tested against
    # the reference's ECS chains (tests/test_gpu_posterior.py).  `value`
    # stays the reference's own sampler.
    alt = None
    if args.method == "ECS" and not args.no_alt:
        sw3 = P.Sweeper(n, P.METHODS["UNIF"], 1, device=local)
        sw3.set_obs(y[lo:hi], cen[lo:hi], obs0=lo)
        sw3.set_global_count(N)
        red3 = None
        if use_coll:
            if in_lib:
                if not attach_rccl(sw3, dist, coll_dev):
                    raise SystemExit("in-library RCCL all-reduce passed its self-test once, then failed it")
            else:
                red3 = make_stats_allreduce(dist, P.stats_len(n), device=coll_dev)
        P.set_seed(20241010)
        w3 = sw3.gibbs(args.warmup + 1, P.METHODS["UNIF"], nu, zeta, T, Cm, zexp, reduce=red3)
        sync()
        t3 = time.perf_counter()
        r3 = sw3.gibbs(args.steps + 1, P.METHODS["UNIF"], nu, zeta, T, Cm, zexp, start=w3[-1], reduce=red3)
        sync()
        dt3 = time.perf_counter() - t3
        k3 = sw3.kernel_ms_total / args.steps
        if dist is not None:
            dt3, k3 = max_over_ranks(dist, [dt3, k3], device=coll_dev)
        if not np.all(np.isfinite(r3)) or sw3.flagged_obs:
            raise SystemExit("UNIF side run: non-finite draws or flagged observations")
        sw3.close()
        alt = {"method": "UNIF", "value": args.steps / dt3, "unit": "iterations/s", "ms_per_step": dt3 / args.steps * 1e3,
               "kernel_ms": k3, "note": "side measurement, same workload and timing as `value`: the opt-in "
                                        "uniformisation sampler (method 8; per-sweep table kernel + sampler "
                                        "kernel), an exact sampler of ECS's conditional path law with no "
                                        "eigendecomposition; posterior-tested against the reference's ECS "
                                        "chains. `value` is the reference's default ECS sampler"}

    weak = None
    if dist is not None and not args.no_weak:
        # Side measurement (not `value`): weak scaling, every rank holding N
        # observations of its own (one chain over world x N observations).
        yw, cw = simulate_ph(S, s, N, seed=DATA_KEY + 1 + rank, censor_frac=args.censor)
        tot = sum_over_ranks(dist, [float(np.sum(yw))], device=coll_dev)[0]
        zexp_w = P.zexp_for(np.array([tot]))
        sw2 = P.Sweeper(n, method, 1, device=local)
        sw2.set_obs(yw, cw, obs0=rank * N)
        sw2.set_global_count(N * world)
        if in_lib and not attach_rccl(sw2, dist, coll_dev):
            raise SystemExit("in-library RCCL all-reduce passed its self-test once, then failed it")
        P.set_seed(20241009)
        warm = sw2.gibbs(args.warmup + 1, method, nu, zeta, T, Cm, zexp_w, reduce=reduce)
        sync()
        t1 = time.perf_counter()
        sw2.gibbs(args.steps + 1, method, nu, zeta, T, Cm, zexp_w, start=warm[-1], reduce=reduce)
        sync()
        dtw = max_over_ranks(dist, [time.perf_counter() - t1], device=coll_dev)[0]
        sw2.close()
        weak = {"N_per_gpu": N, "N_total": N * world, "chain_sweeps_per_s": args.steps / dtw,
                "value": world * args.steps / dtw, "unit": f"{N:.0e}-observation sweeps/s (node)",
                "ms_per_step": dtw / args.steps * 1e3,
                "note": "side measurement: one chain over world x N observations (each rank N of its own); "
                        "value = world x chain sweeps/s; `value` above is the BASELINE metric (strong, N fixed)"}

    if rank == 0:
        # BASELINE.json's configurations by (n, N, censored fraction)
        cfg_name = {(3, 200, 0.0): "cfg1", (5, 10_000, 0.0): "cfg2", (20, 100_000, 0.0): "cfg3",
                    (10, 1_000_000, 0.0): "cfg4", (15, 500_000, 0.3): "cfg5"}.get((n, N, args.censor), "custom")
        sweeps_per_s = args.steps / dt
        local_obs = hi - lo
        achieved = ALG_BYTES_PER_OBS * local_obs / (kernel_ms * 1e-3) / 1e9
        lib_key = P.lib_key()
        traffic, flops, traffic_src = load_counters(args.traffic_file, n, local_obs, args.method, lib_key)
        line = {
            "metric": "Gibbs iterations/sec (whole node), n=10 states × N=1e6 observations",
            "value": sweeps_per_s,
            "unit": "iterations/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": dt / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "f64",
            "data": f"synthetic: N={N} absorption times simulated from BD-exit(n={n}) (pi=e1), "
                    f"censored fraction {args.censor}, Philox key 0x{DATA_KEY:x}",
            "config": {"workload": f"{cfg_name}: phtMCMC2 {args.method}, n={n} states, m={m} parameters, "
                                   f"N={N} obs ({args.censor:.0%} censored), priors nu=1+50*theta, zeta=50, mhit=1",
                       "n": n, "N": N, "method": args.method, "parallelism": f"obs-shard x{world}",
                       "stats_reduce": reduce_note},
            "lib_key": lib_key,
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                         "kernel_ms": kernel_ms, "traffic_source": traffic_src,
                         "note": f"sweep kernel, {ALG_BYTES_PER_OBS} B/obs x {local_obs} obs per launch / "
                                 "HIP-event kernel time; the path is FP64-VALU/latency bound, see roofline_valu"},
        }
        if flops:
            tfs = flops / (kernel_ms * 1e-3) / 1e12
            line["roofline_valu"] = {"bound": "fp64-valu", "achieved": tfs, "peak": FP64_VALU_PEAK_TF,
                                     "unit": "TFLOP/s", "frac": tfs / FP64_VALU_PEAK_TF,
                                     "note": "FP64 lane-flops per launch from PMC (SQ_INSTS_VALU_FLOPS_FP64 x 64 x "
                                             "VALU lane utilisation, profiles/traffic_latest.json) / kernel time"}
        if alt is not None:
            line["alt_sampler"] = alt
        if weak is not None:
            line["weak_scaling"] = weak
        if world == 1 and not args.no_cpu_baseline:
            # UNIF has no reference counterpart: its CPU baseline is the
            # reference's own sampler for the same workload, ECS
            cpu_method = method if method in (1, 2, 4) else 2
            try:
                line["cpu_baseline"] = cpu_baseline(n, y, cen, T, nu, zeta, cpu_method)
            except Exception as e:  # noqa: BLE001
                log(f"[bench] cpu baseline failed: {e}")
                line["cpu_baseline"] = None
            # SURVEY.md §8(d)'s "best CPU" line: the reference on 16 host cores,
            # observations split (a child process: this one has the GPU open)
            try:
                import subprocess

                cmd = [sys.executable, "-m", "oracle.cpu_best", "--n", str(n), "--N", str(N), "--censor",
                       str(args.censor), "--workers", "16", "--seconds", "10", "--method", str(cpu_method)]
                out = subprocess.run(cmd, cwd=REPO, capture_output=True, text=True, timeout=180, check=True).stdout
                line["cpu_best"] = json.loads(out.strip().splitlines()[-1])
                line["cpu_best"]["ratio_gpu_over_cpu_best"] = line["value"] / line["cpu_best"]["value"]
            except Exception as e:  # noqa: BLE001
                log(f"[bench] cpu best line failed: {e}")
                line["cpu_best"] = None
        print(json.dumps(line), flush=True)
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
