#!/bin/bash
# Kernel traces of the UNIF sampler at cfg3 / cfg4 / cfg1 sizes (GPU box).
set -o pipefail
TAG=${1:-unif}
O=$GRAFT_REPO_ROOT/gpurun_out/prof_$TAG; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for cfg in "20 100000" "10 1000000" "3 200"; do set -- $cfg
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/n$1 -o run -- \
    python3 $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline --method UNIF --n $1 --N $2 --steps 20 > $O/n$1.json 2> $O/n$1.err || exit 1
  echo "n=$1 N=$2"; head -4 $O/n$1/run_kernel_stats.csv | cut -c1-150
done
