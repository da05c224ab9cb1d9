#!/bin/bash
# Kernel trace of tools/mhrs_burnin.py --ab I,J (MHRS search rounds per replayed
# chain draw) with the per-round unresolved-task counts (PHT_MHRS_COUNTS=1).
# usage (GPU box): tools/prof_mhrs_ab.sh <tag> I,J
set -o pipefail
TAG=$1; AB=$2
OUT=$GRAFT_REPO_ROOT/gpurun_out/prof_$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
export PHT_MHRS_COUNTS=1
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT -o run -- \
  python3 $GRAFT_REPO_ROOT/tools/mhrs_burnin.py --sweeps 300 --ab $AB > $OUT/ab.out 2> $OUT/ab.err
