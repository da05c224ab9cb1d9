#!/bin/bash
# Interleaved A/B of variant libraries at the ECS configurations, plus the
# ECS parity subset on the default library (GPU box).
# usage: tools/gpu_ab.sh <tag> <lib A> <lib B> [pytest -k expr]
set -o pipefail
TAG=$1; A=$2; B=$3; K=${4:-"bitexact or longest or row_kernel or shard"}
O=$GRAFT_REPO_ROOT/gpurun_out/$TAG; mkdir -p $O; cd $GRAFT_REPO_ROOT
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_edges.py -m gpu -q --timeout 150 --timeout-method thread -k "$K" > $O/pytest.log 2>&1; rc=$?
tail -2 $O/pytest.log; grep -E "FAILED|ERROR" $O/pytest.log | head
[ $rc -le 1 ] || exit $rc
for cfg in "10 1000000 0.0 5" "10 125000 0.0 20" "20 100000 0.0 20" "15 500000 0.3 10" "5 10000 0.0 50"; do set -- $cfg
  timeout -k 10 300 python3 tools/ab.py --libs $A $B --n $1 --N $2 --censor $3 --sweeps $4 --rounds 5 > $O/ab_n$1_N$2.json 2>> $O/ab.err || { tail $O/ab.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/ab_n$1_N$2.json'));print('n=$1 N=$2', {k:(round(v['ms_per_sweep_median'],4),round(v['kernel_ms_median'],4)) for k,v in d.items()} if 'error' not in d else d)"
done
exit $rc
