#!/bin/bash
# cfg5 ECS: rows for the exact range's longest paths, PHT_ROWK = 0 / 128 (default) / 512 / 1024, two rounds
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/${TAG:-r05an}
mkdir -p $O
cd $GRAFT_REPO_ROOT
for r in 1 2; do
  for k in 0 128 512 1024; do
    PHT_ROWK=$k timeout -k 10 200 python3 bench.py --no-cpu-baseline --no-alt --n 15 --N 500000 --censor 0.3 --steps 30 > $O/cfg5_k${k}_$r.json 2>>$O/err.txt || exit 1
  done
  echo round $r
done
python3 - $O <<'PY'
import json, glob, os, sys
for f in sorted(glob.glob(os.path.join(sys.argv[1], "cfg*.json"))):
    d = json.load(open(f)); print(os.path.basename(f), round(d["value"], 1), round(d["ms_per_step"], 4), round(d["roofline"]["kernel_ms"], 4))
PY
