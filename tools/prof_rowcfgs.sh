#!/bin/bash
# rocprofv3 kernel-trace stats at the configs where row blocks run (cfg2,
# cfg3, cfg5 ECS): per-kernel time split.  usage (GPU box): tools/prof_rowcfgs.sh <tag>
set -o pipefail
TAG=${1:-rowprof}
O=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
prof() { local name=$1; shift; timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$name -o run -- python3 $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline "$@" > $O/$name.json 2> $O/$name.err || { echo "$name failed"; exit 1; }; echo "$name ok"; }
prof cfg2_ecs --n 5 --N 10000 --steps 20 --warmup 2
prof cfg3_ecs --n 20 --N 100000 --steps 10 --warmup 2
prof cfg5_ecs --n 15 --N 500000 --censor 0.3 --method ECS --steps 5 --warmup 1
