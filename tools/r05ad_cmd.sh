#!/bin/bash
# cfg2 (n = 5, N = 1e4): rows K (PHT_ROWK) 4096 (default) / 6144 / 8192 / 10000, two rounds of bench.py
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/${TAG:-r05ad}
mkdir -p $O
cd $GRAFT_REPO_ROOT
for r in 1 2; do
  for k in 4096 6144 8192 10000; do
    PHT_ROWK=$k timeout -k 10 200 python3 bench.py --no-cpu-baseline --no-alt --n 5 --N 10000 --steps 300 > $O/cfg2_k${k}_$r.json 2>>$O/err.txt || exit 1
  done
  echo round $r
done
python3 - $O <<'PY'
import json, glob, os, sys
for f in sorted(glob.glob(os.path.join(sys.argv[1], "cfg*.json"))):
    d = json.load(open(f)); print(os.path.basename(f), round(d["value"], 1), round(d["ms_per_step"], 4), round(d["roofline"]["kernel_ms"], 4))
PY
