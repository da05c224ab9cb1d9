set -o pipefail
# exp without the underflow select (clamp at -1100, the ldexp rounds to 0) and with the integer from the
# shifted double's low word: ECS parity subset, then A/B vs HEAD (one process per library)
O=$GRAFT_REPO_ROOT/gpurun_out/r03ab; mkdir -p $O; cd $GRAFT_REPO_ROOT
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_edges.py -m gpu -x -q --timeout 300 --timeout-method thread -k "bitexact or row or cens or shard or state_counts or tiny" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
V=phasetype_amd/_variants
for cfg in "10 1000000 0 10" "10 125000 0 40" "15 500000 0.3 10" "20 100000 0 20" "5 10000 0 50"; do set -- $cfg
  timeout -k 10 400 python3 tools/ab.py --libs $V/base.so $V/lowk0.so phasetype_amd/_lib/libPhaseType.so --method ECS --n $1 --N $2 --censor $3 --sweeps $4 --rounds 5 > $O/ab_$1_$2_$3.json 2> $O/ab_$1_$2_$3.err || { tail $O/ab_$1_$2_$3.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/ab_$1_$2_$3.json'));print('n=$1 N=$2 c=$3', {k.split('/')[-1]:(round(v['ms_per_sweep_median'],4),round(v['kernel_ms_median'],4)) for k,v in d.items()} if 'error' not in d else d)"
done
