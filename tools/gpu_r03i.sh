set -o pipefail
# ECS E0 pre-pass: GPU parity (ECS tests, pre-pass on by default), then bench A/B PHT_E0=0|1 interleaved
O=$GRAFT_REPO_ROOT/gpurun_out/r03i; mkdir -p $O; cd $GRAFT_REPO_ROOT
timeout -k 10 500 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_edges.py tests/test_gpu_posterior.py -m gpu -x -q --timeout 150 --timeout-method thread -k "ECS or ecs or bitexact or longest or row or shard or posterior" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for rep in 1 2; do for e in 0 1; do for cfg in "10 1000000 0 20" "10 125000 0 100" "15 500000 0.3 20" "20 100000 0 50"; do set -- $cfg
  PHT_E0=$e timeout -k 10 200 python3 bench.py --no-cpu-baseline --no-alt --n $1 --N $2 --censor $3 --steps $4 > $O/e${e}_n$1_N$2_r$rep.json 2> $O/e${e}_n$1_N$2_r$rep.err || { tail $O/e${e}_n$1_N$2_r$rep.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/e${e}_n$1_N$2_r$rep.json'));print('E0=$e n=$1 N=$2 rep=$rep', round(d['value'],1), 'ms', round(d['ms_per_step'],4), 'kernel', round(d['roofline']['kernel_ms'],4))"
done; done; done
