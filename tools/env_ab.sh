#!/bin/bash
# bench.py A/B between environment settings (GPU box), interleaved rounds.
# usage: tools/env_ab.sh <tag> "<bench args>" "<env A>" "<env B>" [rounds]
set -o pipefail
TAG=$1; ARGS=$2; EA=$3; EB=$4; R=${5:-3}
O=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $O
cd $GRAFT_REPO_ROOT
for r in $(seq 1 $R); do
  for v in A B; do
    if [ $v = A ]; then E=$EA; else E=$EB; fi
    env $E timeout -k 10 240 python3 bench.py --no-cpu-baseline $ARGS > $O/${v}_$r.json 2> $O/${v}_$r.err || exit 1
    python3 -c "import json; a=json.load(open('$O/${v}_$r.json')); print('$v [$E] round $r', round(a['value'],1), 'sweeps/s', round(a['roofline']['kernel_ms'],3), 'ms')"
  done
done
