#!/bin/bash
# cfg4: new observations per lane per round (PHT_NEWCAP 1 = default, 2, 0 = unlimited), alternating, two rounds
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/${TAG:-r05aj}
mkdir -p $O
cd $GRAFT_REPO_ROOT
for r in 1 2; do
  for k in 1 2 0; do
    PHT_NEWCAP=$k timeout -k 10 200 python3 bench.py --no-cpu-baseline --no-alt --steps 50 > $O/cfg4_nc${k}_$r.json 2>>$O/err.txt || exit 1
  done
  echo round $r
done
python3 - $O <<'PY'
import json, glob, os, sys
for f in sorted(glob.glob(os.path.join(sys.argv[1], "cfg*.json"))):
    d = json.load(open(f)); print(os.path.basename(f), round(d["value"], 1), round(d["ms_per_step"], 4), round(d["roofline"]["kernel_ms"], 4))
PY
