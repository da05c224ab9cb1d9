#!/bin/bash
# One GPU lease, several steps (run on the box via gpurun).  Replaces the
# per-experiment lease scripts of r03 (tools/gpu_r03*.sh): every committed
# profile directory names the gpu_steps.sh command that produced it.
#
# usage: tools/gpu_steps.sh <tag> <step> [<step> ...]
#   tests=<pytest args>      python -m pytest -m gpu <args>  (e.g. tests=tests/test_gpu_fullsize.py)
#   allgpu                   the whole -m gpu suite
#   smoke                    __graft_entry__.smoke()
#   bench=<bench.py args>    one bench line -> bench_<k>.json (k = step index)
#   shards=<W>               tools/latency.py --shards W -> shards_W.jsonl
#   latency=<args>           tools/latency.py <args> -> latency_<k>.jsonl
#   trace=<bench args>       rocprofv3 kernel trace of bench.py (tools/prof_trace.sh)
#   pmc=<bench args>         rocprofv3 PMC passes + summary (tools/prof_pmc.sh, tools/pmc_summary.py)
#   py=<script args>         python3 <script args> -> py_<k>.out
#   configs                  tools/gpu_configs.sh: bench.py at every BASELINE config -> <tag>_cfgs/
#   env=NAME=VALUE           export for the following steps;  unenv=NAME  unset it
# Outputs under gpurun_out/<tag>/; each GPU step has its own time limit and
# the script stops at the first failure (no retries).
set -o pipefail
TAG=$1
shift
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
echo "gpu_steps.sh $TAG $*" > $O/COMMAND
k=0
for step in "$@"; do
  k=$((k + 1))
  name=${step%%=*}
  arg=""
  [[ "$step" == *=* ]] && arg=${step#*=}
  echo "[$k] $step"
  case $name in
    tests)
      timeout -k 10 900 python3 -u -m pytest -m gpu -x -v --timeout 300 --timeout-method thread $arg \
        > $O/pytest_$k.log 2>&1 || { tail -40 $O/pytest_$k.log; exit 1; }
      tail -1 $O/pytest_$k.log ;;
    allgpu)
      timeout -k 10 1100 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
        > $O/pytest_gpu_full.log 2>&1 || { tail -40 $O/pytest_gpu_full.log; exit 1; }
      tail -1 $O/pytest_gpu_full.log ;;
    smoke)
      timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 \
        || { tail -20 $O/smoke.log; exit 1; }
      tail -1 $O/smoke.log ;;
    bench)
      timeout -k 10 600 python3 bench.py $arg > $O/bench_$k.json 2> $O/bench_$k.err \
        || { tail -20 $O/bench_$k.err; exit 1; }
      cat $O/bench_$k.json ;;
    shards)
      timeout -k 10 600 python3 -u tools/latency.py --shards $arg > $O/shards_$arg.jsonl 2> $O/shards_$arg.err \
        || { tail -20 $O/shards_$arg.err; exit 1; }
      tail -1 $O/shards_$arg.jsonl ;;
    latency)
      timeout -k 10 900 python3 -u tools/latency.py $arg > $O/latency_$k.jsonl 2> $O/latency_$k.err \
        || { tail -20 $O/latency_$k.err; exit 1; }
      cat $O/latency_$k.jsonl ;;
    trace)
      bash tools/prof_trace.sh ${TAG}_$k $arg || { echo "trace failed"; exit 1; }
      cp $R/gpurun_out/prof_${TAG}_$k/run_kernel_stats.csv $O/trace_${k}_kernel_stats.csv 2>/dev/null
      head -8 $O/trace_${k}_kernel_stats.csv | cut -d, -f1-4 ;;
    pmc)
      bash tools/prof_pmc.sh ${TAG}_$k $arg || { echo "pmc failed"; exit 1; }
      python3 tools/pmc_summary.py $R/gpurun_out/pmc_${TAG}_$k $O/pmc_${k}_summary.json $O/pmc_${k}_traffic.json \
        > $O/pmc_${k}_summary.out 2>&1 || { tail $O/pmc_${k}_summary.out; exit 1; }
      tail -25 $O/pmc_${k}_summary.out ;;
    env)
      export "$arg" ;;
    unenv)
      unset "$arg" ;;
    configs)
      bash tools/gpu_configs.sh ${TAG}_cfgs || { echo "configs failed"; exit 1; }
      cp $R/gpurun_out/${TAG}_cfgs/*.json $O/ 2>/dev/null ;;
    py)
      timeout -k 10 900 python3 -u $arg > $O/py_$k.out 2> $O/py_$k.err || { tail -20 $O/py_$k.err; exit 1; }
      tail -5 $O/py_$k.out ;;
    *)
      echo "unknown step $step"; exit 2 ;;
  esac
done
echo "all steps ok"
