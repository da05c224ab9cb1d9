#!/bin/bash
# GPU tests, row stamps (top64), shard-size latency and all configs.
# usage (GPU box): tools/gpu_rowcheck.sh <tag>
set -o pipefail
TAG=${1:-rowcheck}
O=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $O
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { echo "gpu tests failed"; tail -30 $O/pytest.log; exit 1; }
echo "gpu tests ok"
PHT_LIB=phasetype_amd/_variants/stamps.so PHT_ROWK=64 timeout -k 10 120 python3 tools/stamps.py --top 64 > $O/stamps_row64.json 2>&1 || exit 1
timeout -k 10 300 python3 tools/latency.py --Ns top64 31250 62500 125000 250000 --variants base row0 --sweeps 6 > $O/lat.jsonl 2> $O/lat.err || exit 1
echo "latency ok"
bash tools/gpu_configs.sh ${TAG}_cfg
