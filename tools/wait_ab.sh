#!/bin/bash
# Host wait mode A/B (GPU box): bench.py with the HIP runtime's default wait
# against ROC_ACTIVE_WAIT_TIMEOUT=<T> (busy-wait before sleeping), alternating
# processes.  usage: tools/wait_ab.sh <tag> <T>
set -o pipefail
TAG=${1:-wait}; T=${2:-5000}
O=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $O
cd $GRAFT_REPO_ROOT
for rep in 1 2; do
  for cfg in "10 1000000 20" "10 125000 100" "5 10000 200"; do
    set -- $cfg
    for mode in def spin; do
      if [ $mode = spin ]; then export ROC_ACTIVE_WAIT_TIMEOUT=$T; else unset ROC_ACTIVE_WAIT_TIMEOUT; fi
      timeout -k 10 120 python3 bench.py --no-cpu-baseline --n $1 --N $2 --steps $3 --warmup 3 > $O/${mode}_n$1_N$2_$rep.json 2> $O/${mode}_n$1_N$2_$rep.err || exit 1
      python3 -c "import json; a=json.load(open('$O/${mode}_n$1_N$2_$rep.json')); print('$mode n=$1 N=$2 rep $rep', round(a['ms_per_step'],4), 'ms/step', round(a['roofline']['kernel_ms'],4), 'kernel ms')"
    done
  done
done
