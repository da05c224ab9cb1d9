set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r03e; mkdir -p $O; cd $GRAFT_REPO_ROOT
for N in 1000000 125000; do
  PHT_LIB=phasetype_amd/_variants/diag.so timeout -k 10 120 python3 tools/ecs_diag.py --N $N >> $O/diag.jsonl 2>> $O/diag.err || { tail $O/diag.err; exit 1; }
done
cat $O/diag.jsonl
timeout -k 10 300 python3 bench.py > $O/bench.json 2> $O/bench.err || { tail $O/bench.err; exit 1; }
cat $O/bench.json
bash tools/prof_trace.sh r03e --steps 10 || { echo "trace failed"; exit 1; }
bash tools/prof_pmc.sh r03e --steps 5 --warmup 1 || { echo "pmc failed"; exit 1; }
python3 tools/pmc_summary.py $GRAFT_REPO_ROOT/gpurun_out/pmc_r03e $O/pmc_summary.json $O/traffic.json > /dev/null && echo pmc ok
