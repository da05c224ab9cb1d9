#!/bin/bash
# PHT_PARAMS_HOST=1 (kernels read the parameter block from pinned host memory, no per-sweep copy) against the
# default: parity + chain tests under it, then bench.py alternating at cfg1 / cfg2 / cfg4, two rounds
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/${TAG:-r05ab}
mkdir -p $O
cd $GRAFT_REPO_ROOT
PHT_PARAMS_HOST=1 timeout -k 10 500 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_edges.py > $O/tests.txt 2>&1 && echo tests ok || { tail -30 $O/tests.txt; exit 1; }
b() { timeout -k 10 200 python3 bench.py --no-cpu-baseline --no-alt "$@"; }
for r in 1 2; do
  b --n 3 --N 200 --steps 1000 > $O/cfg1_dev_$r.json 2>>$O/err.txt &&
  PHT_PARAMS_HOST=1 b --n 3 --N 200 --steps 1000 > $O/cfg1_host_$r.json 2>>$O/err.txt &&
  b --n 5 --N 10000 --steps 200 > $O/cfg2_dev_$r.json 2>>$O/err.txt &&
  PHT_PARAMS_HOST=1 b --n 5 --N 10000 --steps 200 > $O/cfg2_host_$r.json 2>>$O/err.txt &&
  b --steps 50 > $O/cfg4_dev_$r.json 2>>$O/err.txt &&
  PHT_PARAMS_HOST=1 b --steps 50 > $O/cfg4_host_$r.json 2>>$O/err.txt && echo round $r || exit 1
done
python3 - $O <<'PY'
import json, glob, os, sys
for f in sorted(glob.glob(os.path.join(sys.argv[1], "cfg*.json"))):
    d = json.load(open(f)); print(os.path.basename(f), round(d["value"], 1), round(d["ms_per_step"], 4), round(d["roofline"]["kernel_ms"], 4))
PY
