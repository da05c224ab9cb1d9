#!/bin/bash
# bench.py at every BASELINE.json config that fits one GPU (no CPU baseline):
# cfg1 n=3 N=200 ECS (the CPU-plumbing config, 1000 sweeps); cfg2 n=5 N=1e4 ECS; cfg3 n=20 N=1e5 ECS; cfg4 n=10 N=1e6 ECS + MHRS;
# cfg5 n=15 N=5e5 30% censored, MHRS / DCS / ECS.  MHRS runs 100 sweeps: its per-sweep cost follows
# the current draw of the slowest decay rate (the hardest observations need ~e^{delta y} attempts),
# so short runs scatter widely.  usage: tools/gpu_configs.sh <tag>
set -o pipefail
TAG=${1:-cfgs}
O=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $O
cd $GRAFT_REPO_ROOT
run() { local name=$1; shift; timeout -k 10 240 python3 bench.py --no-cpu-baseline "$@" > $O/$name.json 2> $O/$name.err || { echo "$name failed"; exit 1; }; echo "$name ok"; }
run cfg1_ecs --n 3 --N 200 --steps 1000
run cfg2_ecs --n 5 --N 10000 --steps 50
run cfg3_ecs --n 20 --N 100000 --steps 20
run cfg4_ecs --n 10 --N 1000000 --steps 20
run cfg4_mhrs --n 10 --N 1000000 --method MHRS --steps 100
run cfg5_mhrs --n 15 --N 500000 --censor 0.3 --method MHRS --steps 100
# past burn-in (MHRS's attempt count follows the draw: profiles/r04/steady/)
run cfg4_mhrs_steady --n 10 --N 1000000 --method MHRS --warmup 200 --steps 100
run cfg5_mhrs_steady --n 15 --N 500000 --censor 0.3 --method MHRS --warmup 200 --steps 100
run cfg5_dcs --n 15 --N 500000 --censor 0.3 --method DCS --steps 50
run cfg5_ecs --n 15 --N 500000 --censor 0.3 --method ECS --steps 20
run cfg3_unif --n 20 --N 100000 --method UNIF --steps 50
run cfg5_unif --n 15 --N 500000 --censor 0.3 --method UNIF --steps 20
python3 - $O <<'PY'
import json, sys, glob, os
for f in sorted(glob.glob(os.path.join(sys.argv[1], "cfg*.json"))):
    d = json.load(open(f))
    alt = d.get("alt_sampler") or {}
    print(f"{os.path.basename(f)[:-5]:12s} {d['value']:9.1f} sweeps/s  ms/step {d['ms_per_step']:.4f}  kernel {d['roofline']['kernel_ms']:.4f}"
          + (f"  | UNIF {alt['value']:.1f}" if alt else ""))
PY
