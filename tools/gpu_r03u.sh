set -o pipefail
# DCS end-state pre-pass: full GPU suite, then interleaved A/B against HEAD
O=$GRAFT_REPO_ROOT/gpurun_out/r03u; mkdir -p $O; cd $GRAFT_REPO_ROOT
timeout -k 10 1100 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu_full.log 2>&1 || { tail -40 $O/pytest_gpu_full.log; exit 1; }
tail -1 $O/pytest_gpu_full.log
for cfg in "15 500000 0.3 10" "10 1000000 0 5" "20 100000 0 20" "5 10000 0 50" "3 200 0 200"; do set -- $cfg
  timeout -k 10 400 python3 tools/ab.py --libs phasetype_amd/_variants/base.so phasetype_amd/_lib/libPhaseType.so --method DCS --n $1 --N $2 --censor $3 --sweeps $4 --rounds 4 > $O/ab_n$1.json 2> $O/ab_n$1.err || { tail $O/ab_n$1.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/ab_n$1.json'));print('n=$1 N=$2 c=$3', {k.split('/')[-1]:(round(v['ms_per_sweep_median'],4),round(v['kernel_ms_median'],4)) for k,v in d.items()} if 'error' not in d else d)"
done
