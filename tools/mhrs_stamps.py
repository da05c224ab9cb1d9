#!/usr/bin/env python3
"""Where an MHRS search wavefront's cycles go (r06): the refill code (item
claim, the item's y / gid / cens loads, stream init) against the rest of the
iteration (start state, Philox top-up, one jump, record check), from a
-D PHT_MHRS_STAMPS variant build (PHT_LIB; diagnostic, never timed).

Runs a cfg4-shaped fresh MHRS chain (tools/mhrs_burnin.py's set-up) with the
product library to get its parameter draws, then replays single sweeps at
draws of the fresh window and of the steady state with the stamps library.

usage (GPU box): python3 tools/mhrs_stamps.py --lib phasetype_amd/_variants/mstamp.so [--sweeps 40]
"""
import argparse
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--lib", required=True)
    ap.add_argument("--sweeps", type=int, default=240)
    ap.add_argument("--at", default="5,20,60,230")
    ap.add_argument("--n", type=int, default=10)
    ap.add_argument("--N", type=int, default=1_000_000)
    a = ap.parse_args()
    os.environ["PHT_LIB"] = os.path.abspath(a.lib)
    import phasetype_amd as P
    from phasetype_amd.synth import DATA_KEY, bd_exit, bd_exit_structure, simulate_ph
    from mhrs_burnin import generator

    n = a.n
    S0, s0 = bd_exit(n)
    T, theta = bd_exit_structure(n)
    nu, zeta = 1.0 + 50.0 * theta, np.full(len(theta), 50.0)
    y, cen = simulate_ph(S0, s0, a.N, seed=DATA_KEY)
    zexp = P.zexp_for(y)
    sw = P.Sweeper(n, P.METHODS["MHRS"], 1)
    sw.set_obs(y, cen)
    P.set_seed(20241008)
    res = sw.gibbs(a.sweeps + 1, P.METHODS["MHRS"], nu, zeta, T, np.ones(T.shape), zexp)
    for it in (int(v) for v in a.at.split(",")):
        S, s = generator(res[it], T, n)
        st = sw.sweep(S, s, key=(11, 13), sweep=it + 1, zexp=zexp)
        ex = [float(v) for v in P.split_stats(st, n)[3]]
        ref, rest, wit, cref, cit, ref0, all0 = ex[8:15]
        tot = ref + rest
        print(json.dumps({"sweep": it, "kernel_ms": sw.last_kernel_ms(), "wave_iters": int(wit),
                          "refill_share": ref / tot, "cycles_per_wave_iter": tot / max(1.0, wit),
                          "refill_cycles_per_wave_iter": ref / max(1.0, wit),
                          "claim_iter_share": cit / max(1.0, wit),
                          "refill_cycles_per_claim_iter": cref / max(1.0, cit),
                          "refill_cycles_per_other_iter": (ref - cref) / max(1.0, wit - cit),
                          "round0_share_of_cycles": all0 / tot, "round0_refill_share": ref0 / max(1.0, all0)}),
              flush=True)
    sw.close()


if __name__ == "__main__":
    main()
