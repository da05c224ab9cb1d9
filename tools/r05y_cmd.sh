#!/bin/bash
# host-side timeline of the cfg4 bench: HIP runtime API + kernel + memory-copy traces (no counters)
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/${TAG:-r05y}
mkdir -p $O
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --hip-runtime-trace --kernel-trace --memory-copy-trace --output-format csv -d $O/trace -o run -- python3 bench.py --steps 30 --no-cpu-baseline --no-alt > $O/bench.json 2>$O/bench.err && echo trace
