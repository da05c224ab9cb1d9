#!/bin/bash
# Full GPU check for a round (run on the box via gpurun):
#   GPU parity tests, smoke(), default bench line (with cpu_baseline),
#   rocprofv3 kernel trace + PMC passes, summaries into gpurun_out/.
# usage: tools/gpu_round.sh <tag>
set -o pipefail
TAG=${1:-r01}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
timeout -k 10 600 python3 -m pytest tests -m gpu -x -q > $O/pytest_gpu.log 2>&1 || { echo "gpu tests failed"; exit 1; }
echo "gpu tests ok"
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke failed"; exit 1; }
echo "smoke ok"
timeout -k 10 600 python3 bench.py > $O/bench.json 2> $O/bench.err || { echo "bench failed"; exit 1; }
echo "bench ok"
bash tools/prof_trace.sh $TAG --steps 10 || { echo "trace failed"; exit 1; }
echo "trace ok"
bash tools/prof_pmc.sh $TAG --steps 5 --warmup 1 || { echo "pmc failed"; exit 1; }
cd $R && python3 tools/pmc_summary.py $R/gpurun_out/pmc_$TAG $O/pmc_summary.json $O/traffic.json > /dev/null
echo "pmc ok"
