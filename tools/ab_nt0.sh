#!/bin/bash
# A/B: per-n compiled kernels vs the runtime-n kernels (PHT_FORCE_NT0=1) at cfg5 DCS / ECS and cfg3 ECS
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/abnt0
mkdir -p $O; cd $GRAFT_REPO_ROOT
b() { timeout -k 10 200 python3 bench.py --no-cpu-baseline "$@"; }
for r in 1 2; do
b --n 15 --N 500000 --censor 0.3 --method DCS --steps 4 > $O/dcs_nt$r.json 2>/dev/null || exit 1
PHT_FORCE_NT0=1 b --n 15 --N 500000 --censor 0.3 --method DCS --steps 4 > $O/dcs_g$r.json 2>/dev/null || exit 1
done
b --n 15 --N 500000 --censor 0.3 --method ECS --steps 8 > $O/ecs5_nt.json 2>/dev/null || exit 1
PHT_FORCE_NT0=1 b --n 15 --N 500000 --censor 0.3 --method ECS --steps 8 > $O/ecs5_g.json 2>/dev/null || exit 1
b --n 20 --N 100000 --steps 20 > $O/ecs3_nt.json 2>/dev/null || exit 1
PHT_FORCE_NT0=1 b --n 20 --N 100000 --steps 20 > $O/ecs3_g.json 2>/dev/null || exit 1
for f in $O/*.json; do python3 -c "import json; d=json.load(open('$f')); print('$(basename $f)', round(d['value'],1), round(d['roofline']['kernel_ms'],3))"; done
