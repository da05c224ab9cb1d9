#!/bin/bash
# DCS kernel A/B on cfg5-shaped data (GPU box): GPU tests, then bench.py
# with the one-lane legacy kernel (PHT_DCS_LEGACY=1), the jump-converged
# kernel, and optional variant libraries (PHT_LIB).  usage: tools/dcs_ab.sh <tag> [variant.so ...]
set -o pipefail
TAG=${1:-dcs}; shift
O=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $O
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
b() { timeout -k 10 240 python3 bench.py --no-cpu-baseline --n $1 --N 500000 --censor 0.3 --method DCS --steps 5 > $O/$2_n$1.json 2> $O/$2_n$1.err || exit 1;
      python3 -c "import json; a=json.load(open('$O/$2_n$1.json')); print('n=$1 $2', round(a['value'],1), 'sweeps/s', round(a['roofline']['kernel_ms'],3), 'ms')"; }
for n in 10 15; do
  PHT_DCS_LEGACY=1 b $n legacy
  b $n round
  for v in "$@"; do PHT_LIB=$v b $n $(basename $v .so); done
done
