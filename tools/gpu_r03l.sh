set -o pipefail
# DCS by the Halley root: GPU parity (DCS cases, Brent mode, chains, posterior), then bench A/B vs PHT_DCS_ROOT=brent
O=$GRAFT_REPO_ROOT/gpurun_out/r03l; mkdir -p $O; cd $GRAFT_REPO_ROOT
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_posterior.py tests/test_gpu_resident.py -m gpu -x -q --timeout 300 --timeout-method thread -k "dcs or DCS or -4- or 4-5 or 4-4 or 4-3 or chains or brent" > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for r in halley brent; do for cfg in "15 500000 0.3 10" "10 1000000 0 5" "5 10000 0 50"; do set -- $cfg
  if [ $r = brent ]; then export PHT_DCS_ROOT=brent; else unset PHT_DCS_ROOT; fi
  timeout -k 10 240 python3 bench.py --no-cpu-baseline --no-alt --method DCS --n $1 --N $2 --censor $3 --steps $4 > $O/${r}_n$1.json 2> $O/${r}_n$1.err || { tail $O/${r}_n$1.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/${r}_n$1.json'));print('$r n=$1 N=$2', round(d['value'],1), 'ms', round(d['ms_per_step'],4), 'kernel', round(d['roofline']['kernel_ms'],4))"
done; done
