#!/bin/bash
# statistics published by the ECS exact launch's last block (single-launch sweeps) against HEAD (a separate
# publishing kernel): the whole GPU suite, then bench.py alternating at cfg1 / cfg2 / cfg4, two rounds
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/${TAG:-r05ah}
mkdir -p $O
cd $GRAFT_REPO_ROOT
H=phasetype_amd/_variants/head.so
timeout -k 10 1000 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu_full.log 2>&1 && tail -1 $O/pytest_gpu_full.log || { tail -30 $O/pytest_gpu_full.log; exit 1; }
b() { timeout -k 10 200 python3 bench.py --no-cpu-baseline --no-alt "$@"; }
for r in 1 2; do
  PHT_LIB=$H b --n 3 --N 200 --steps 1000 > $O/cfg1_head_$r.json 2>>$O/err.txt &&
  b --n 3 --N 200 --steps 1000 > $O/cfg1_new_$r.json 2>>$O/err.txt &&
  PHT_LIB=$H b --n 5 --N 10000 --steps 300 > $O/cfg2_head_$r.json 2>>$O/err.txt &&
  b --n 5 --N 10000 --steps 300 > $O/cfg2_new_$r.json 2>>$O/err.txt &&
  PHT_LIB=$H b --steps 50 > $O/cfg4_head_$r.json 2>>$O/err.txt &&
  b --steps 50 > $O/cfg4_new_$r.json 2>>$O/err.txt && echo round $r || exit 1
done
python3 - $O <<'PY'
import json, glob, os, sys
for f in sorted(glob.glob(os.path.join(sys.argv[1], "cfg*.json"))):
    d = json.load(open(f)); print(os.path.basename(f), round(d["value"], 1), round(d["ms_per_step"], 4), round(d["roofline"]["kernel_ms"], 4))
PY
