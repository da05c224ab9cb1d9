#!/usr/bin/env python3
"""Per-phase cycle breakdown (wave-level s_memtime stamps; the stats block's
extra words carry [rounds, 15 stamp slots] in PHT_STAMPS builds) of the ECS exact kernel from a PHT_STAMPS build
(diagnostic only: stamps perturb the schedule; read shares, not totals).
usage: PHT_LIB=/path/variant.so python3 tools/stamps.py [--N 1000000]"""
import argparse
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import phasetype_amd as P  # noqa: E402
from phasetype_amd.synth import DATA_KEY, bd_exit, simulate_ph  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--n", type=int, default=10)
ap.add_argument("--N", type=int, default=1_000_000)
ap.add_argument("--top", type=int, default=0, help="only the TOP largest observations (lone-wave latency)")
a = ap.parse_args()
S, s = bd_exit(a.n)
y, cen = simulate_ph(S, s, a.N, seed=DATA_KEY)
if a.top:
    idx = np.sort(np.argsort(-y)[:a.top])
    y, cen = np.ascontiguousarray(y[idx]), np.ascontiguousarray(cen[idx])
    a.N = a.top
sw = P.Sweeper(a.n, 2)
sw.set_obs(y, cen)
zexp = P.zexp_for(y)
sw.sweep(S, s, zexp=zexp)
st = sw.sweep(S, s, key=(3, 4), zexp=zexp)
ex = st[2 * a.n + a.n * a.n:]
names = ["phaseA_absorb_newobs", "dens_load_E0", "start_init4", "pend_insert", "meets", "cumulate", "f0_cap",
         "invert_u", "proposal_eval", "test_metropolis", "big_general", "finish_movemass", "topup"]
rounds = float(ex[0])
cyc = [float(v) for v in ex[1:1 + len(names)]]
tot = sum(cyc)
print(json.dumps({"kernel_ms": sw.last_kernel_ms(), "N": a.N, "wave_rounds": rounds,
                  "cycles_per_wave_round": round(tot / max(rounds, 1), 1),
                  "cycles_per_round": {k: round(v / max(rounds, 1), 1) for k, v in zip(names, cyc)},
                  "shares": {k: round(v / tot, 4) for k, v in zip(names, cyc)}}, indent=1))
