#!/bin/bash
# rocprofv3 kernel-trace stats of bench.py at the non-default configs
# (per-kernel time split).  usage (GPU box): tools/prof_cfgs.sh <tag>
set -o pipefail
TAG=${1:-cfgprof}
O=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
prof() { local name=$1; shift; timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$name -o run -- python3 $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline "$@" > $O/$name.json 2> $O/$name.err || { echo "$name failed"; exit 1; }; echo "$name ok"; }
prof cfg4_mhrs --n 10 --N 1000000 --method MHRS --steps 5 --warmup 1
prof cfg5_dcs --n 15 --N 500000 --censor 0.3 --method DCS --steps 3 --warmup 1
prof cfg5_ecs --n 15 --N 500000 --censor 0.3 --method ECS --steps 5 --warmup 1
