set -o pipefail
# censored ECS LDS envelope, re-measured with one process per library: ECS parity subset, then A/B vs HEAD
O=$GRAFT_REPO_ROOT/gpurun_out/r03y; mkdir -p $O; cd $GRAFT_REPO_ROOT
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_edges.py -m gpu -x -q --timeout 300 --timeout-method thread -k "bitexact or cens or chains or shard or state_counts or tiny" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for cfg in "15 500000 0.3 10" "10 1000000 0.3 10" "20 500000 0.3 10" "5 1000000 0.3 20" "10 1000000 0 10"; do set -- $cfg
  timeout -k 10 400 python3 tools/ab.py --libs phasetype_amd/_variants/base.so phasetype_amd/_lib/libPhaseType.so --method ECS --n $1 --N $2 --censor $3 --sweeps $4 --rounds 5 > $O/ab_$1_$2_$3.json 2> $O/ab_$1_$2_$3.err || { tail $O/ab_$1_$2_$3.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/ab_$1_$2_$3.json'));print('n=$1 N=$2 c=$3', {k.split('/')[-1]:(round(v['ms_per_sweep_median'],4),round(v['kernel_ms_median'],4)) for k,v in d.items()} if 'error' not in d else d)"
done
