#!/bin/bash
# Kernel-trace profile of bench.py (run on the GPU box via gpurun).
# usage: tools/prof_trace.sh <tag> [bench args...]
set -o pipefail
TAG=$1; shift
OUT=$GRAFT_REPO_ROOT/gpurun_out/prof_$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT -o run -- \
  python3 $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline --no-alt "$@" > $OUT/bench.json 2> $OUT/bench.err
