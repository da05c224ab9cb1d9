set -o pipefail
# MHRS: round-0 record-load skip, interleaved A/B against HEAD (base.so) + MHRS parity tests
O=$GRAFT_REPO_ROOT/gpurun_out/r03m; mkdir -p $O; cd $GRAFT_REPO_ROOT
timeout -k 10 500 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread -k "MHRS or mhrs or -1-1 or -1-4 or -1-2 or chains" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for cfg in "15 500000 0.3 20" "10 1000000 0 10"; do set -- $cfg
  timeout -k 10 400 python3 tools/ab.py --libs phasetype_amd/_variants/base.so phasetype_amd/_lib/libPhaseType.so --method MHRS --n $1 --N $2 --censor $3 --sweeps $4 --rounds 4 > $O/ab_n$1.json 2> $O/ab_n$1.err || { tail $O/ab_n$1.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/ab_n$1.json'));print('n=$1', {k.split('/')[-1]:(round(v['ms_per_sweep_median'],4),round(v['kernel_ms_median'],4)) for k,v in d.items()} if 'error' not in d else d)"
done
