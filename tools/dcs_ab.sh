#!/bin/bash
# DCS kernel A/B on cfg5-shaped data (GPU box): the GPU tests with every
# DCS kernel (PHT_DCS_KERNEL = legacy | jump), then bench.py with each.
# usage: tools/dcs_ab.sh <tag> [n ...]
set -o pipefail
TAG=${1:-dcs}; shift
NS=${@:-10 15}
O=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $O
cd $GRAFT_REPO_ROOT
for k in jump; do
  PHT_DCS_KERNEL=$k timeout -k 10 400 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_$k.log 2>&1 || { tail -30 $O/pytest_$k.log; exit 1; }
  echo "$k: $(tail -1 $O/pytest_$k.log)"
done
for n in $NS; do
  for k in legacy jump; do
    PHT_DCS_KERNEL=$k timeout -k 10 240 python3 bench.py --no-cpu-baseline --n $n --N 500000 --censor 0.3 --method DCS --steps 5 > $O/${k}_n$n.json 2> $O/${k}_n$n.err || exit 1
    python3 -c "import json; a=json.load(open('$O/${k}_n$n.json')); print('n=$n $k', round(a['value'],1), 'sweeps/s', round(a['roofline']['kernel_ms'],3), 'ms')"
  done
done
