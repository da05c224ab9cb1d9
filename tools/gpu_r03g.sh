set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r03g; mkdir -p $O; cd $GRAFT_REPO_ROOT
for a in 0 1; do for cfg in "20 100000" "10 1000000" "15 500000"; do set -- $cfg
  PHT_UNIF_ALDS=$a timeout -k 10 200 python3 bench.py --no-cpu-baseline --method UNIF --n $1 --N $2 --steps 30 > $O/alds${a}_n$1.json 2> $O/alds${a}_n$1.err || { tail $O/alds${a}_n$1.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/alds${a}_n$1.json'));print('ALDS=$a n=$1', round(d['value'],1), 'kernel', round(d['roofline']['kernel_ms'],4))"
done; done
cd /tmp && export TMPDIR=/tmp
for m in MHRS DCS; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/tr_$m -o run -- python3 $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline --no-alt --n 15 --N 500000 --censor 0.3 --method $m --steps 5 > $O/tr_$m.json 2> $O/tr_$m.err || exit 1
  echo $m; head -16 $O/tr_$m/run_kernel_stats.csv | cut -d, -f1-4
done
