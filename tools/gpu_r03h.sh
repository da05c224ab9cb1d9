set -o pipefail
# UNIF bridge v2: GPU parity (UNIF / resident / chains tests) then the UNIF bench configs
O=$GRAFT_REPO_ROOT/gpurun_out/r03h; mkdir -p $O; cd $GRAFT_REPO_ROOT
timeout -k 10 400 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "unif or UNIF or resident or chains" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for cfg in "20 100000 0" "10 1000000 0" "15 500000 0" "15 500000 0.3"; do set -- $cfg
  timeout -k 10 200 python3 bench.py --no-cpu-baseline --method UNIF --n $1 --N $2 --censor $3 --steps 30 > $O/unif_n$1_c$3.json 2> $O/unif_n$1_c$3.err || { tail $O/unif_n$1_c$3.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/unif_n$1_c$3.json'));print('n=$1 N=$2 cens=$3', round(d['value'],1), 'kernel', round(d['roofline']['kernel_ms'],4))"
done
