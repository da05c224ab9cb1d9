set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r03b; mkdir -p $O; cd $GRAFT_REPO_ROOT
timeout -k 10 600 python3 -u -m pytest tests -m gpu -v --timeout 150 --timeout-method thread -k "unif or hardening or contexts or processed or overflow" > $O/pytest.log 2>&1; rc=$?
tail -3 $O/pytest.log; grep -E "FAILED|ERROR" $O/pytest.log | head -20
[ $rc -le 1 ] || exit $rc
for cfg in "20 100000" "10 1000000" "5 10000"; do set -- $cfg
  timeout -k 10 300 python3 bench.py --no-cpu-baseline --method UNIF --n $1 --N $2 --steps 20 > $O/unif_n$1.json 2> $O/unif_n$1.err || { tail $O/unif_n$1.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/unif_n$1.json'));print('UNIF n=$1 N=$2', round(d['value'],1),'sweeps/s', 'kernel ms',round(d['roofline']['kernel_ms'],4),'ms/step',round(d['ms_per_step'],4))"
done
