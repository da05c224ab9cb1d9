#!/bin/bash
# GPU parity suite + smoke + a short bench line (run on the box via gpurun).
# usage: tools/gpu_check.sh <tag> [pytest -k expression]
set -o pipefail
TAG=${1:-check}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
K=()
[ -n "$2" ] && K=(-k "$2")
timeout -k 10 900 python3 -u -m pytest tests -m gpu -v --timeout 150 --timeout-method thread "${K[@]}" > $O/pytest_gpu.log 2>&1
rc=$?
tail -5 $O/pytest_gpu.log
grep -E "FAILED|ERROR" $O/pytest_gpu.log | head -30
[ $rc -eq 0 ] || [ $rc -eq 1 ] || { echo "pytest rc=$rc (abort/timeout)"; exit $rc; }
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke failed"; cat $O/smoke.log | tail; exit 1; }
echo "smoke ok"
timeout -k 10 600 python3 bench.py --steps 10 > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail $O/bench.err; exit 1; }
echo "bench ok"; cat $O/bench.json
exit $rc
