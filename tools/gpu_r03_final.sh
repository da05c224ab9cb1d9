set -o pipefail
# Round-end evidence (r03): full GPU suite, smoke, default bench, kernel trace,
# PMC passes + traffic summary.  Each GPU step under its own time limit;
# the script stops at the first failure.
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r03final; mkdir -p $O; cd $R
timeout -k 10 1100 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu_full.log 2>&1 || { tail -40 $O/pytest_gpu_full.log; exit 1; }
tail -1 $O/pytest_gpu_full.log
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 400 python3 bench.py > $O/bench_default.json 2> $O/bench_default.err || { tail -20 $O/bench_default.err; exit 1; }
cat $O/bench_default.json
bash tools/prof_trace.sh r03final --steps 20 || exit 1
head -12 $R/gpurun_out/prof_r03final/run_kernel_stats.csv | cut -d, -f1-4
bash tools/prof_pmc.sh r03final --steps 5 || exit 1
python3 tools/pmc_summary.py $R/gpurun_out/pmc_r03final $O/pmc_summary.json $O/traffic_latest.json > $O/pmc_summary.out 2>&1 || { tail $O/pmc_summary.out; exit 1; }
tail -25 $O/pmc_summary.out
