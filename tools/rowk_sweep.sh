#!/bin/bash
# bench.py kernel time at the ECS configs for several PHT_ROWK values
# (the K longest exact observations on 16-lane rows).
# usage (GPU box): tools/rowk_sweep.sh <tag> [K ...]
set -o pipefail
TAG=${1:-rowk}; shift
KS=${@:-0 64 256 1024 2048}
O=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $O
cd $GRAFT_REPO_ROOT
for K in $KS; do
  for cfg in "cfg2 --n 5 --N 10000 --steps 50" "cfg4 --n 10 --N 1000000 --steps 20" "cfg4h --n 10 --N 500000 --steps 20" "cfg5 --n 15 --N 500000 --censor 0.3 --steps 10"; do
    set -- $cfg; name=$1; shift
    PHT_ROWK=$K timeout -k 10 240 python3 bench.py --no-cpu-baseline "$@" > $O/${name}_k$K.json 2> $O/${name}_k$K.err || { echo "$name k$K failed"; exit 1; }
  done
  echo "k$K ok"
done
