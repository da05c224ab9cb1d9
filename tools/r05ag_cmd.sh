#!/bin/bash
# MHRS finish with the next observation prefetched: parity, then the finish kernel's duration in a kernel trace
# of the cfg4 MHRS bench, HEAD (head.so) and the working tree, alternating twice; and ab.py on the sweep
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/${TAG:-r05ag}
mkdir -p $O
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
H=phasetype_amd/_variants/head.so; N=phasetype_amd/_lib/libPhaseType.so
timeout -k 10 500 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_edges.py > $O/tests.txt 2>&1 && echo tests ok || { tail -30 $O/tests.txt; exit 1; }
for r in 1 2; do
  for v in head new; do
    L=$H; [ $v = new ] && L=$N
    PHT_LIB=$L timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/tr_${v}_$r -o run -- python3 bench.py --method MHRS --steps 20 --no-cpu-baseline --no-alt > $O/bench_${v}_$r.json 2>>$O/err.txt || exit 1
  done
  echo round $r
done
timeout -k 10 300 python3 tools/ab.py --libs $H $N --method MHRS --rounds 5 --sweeps 10 > $O/ab_cfg4.json && echo ab
