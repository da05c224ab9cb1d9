#!/bin/bash
# chains check on the box: parity tests of pht_gibbs_run_chains (one launch and
# per-stream), then throughput for both launch modes.  usage: tools/gpu_chains.sh <tag>
set -o pipefail
TAG=${1:-chains}
O=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $O
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py -k chains -x -v --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 300 python3 tools/chains.py --Ks 1 2 4 8 12 16 --cfgs cfg1:3:200:ECS cfg2:5:10000:ECS cfg3:20:100000:ECS > $O/one.jsonl 2> $O/one.err || { tail $O/one.err; exit 1; }
PHT_CHAINS_LAUNCH=streams timeout -k 10 300 python3 tools/chains.py --Ks 1 4 8 12 --cfgs cfg2:5:10000:ECS > $O/streams.jsonl 2> $O/streams.err || exit 1
cat $O/one.jsonl $O/streams.jsonl
