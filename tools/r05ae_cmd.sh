#!/bin/bash
# cfg5 ECS: censored-range grid at 1 block per CU (PHT_CENS_OCC=1, co-resident with the exact kernel's 1 block per
# CU) against the default (its own occupancy, 2 per CU: half its blocks wait for a slot); also n = 10, 30 % censored
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/${TAG:-r05ae}
mkdir -p $O
cd $GRAFT_REPO_ROOT
b() { timeout -k 10 200 python3 bench.py --no-cpu-baseline --no-alt "$@"; }
for r in 1 2 3; do
  b --n 15 --N 500000 --censor 0.3 --steps 30 > $O/cfg5_def_$r.json 2>>$O/err.txt &&
  PHT_CENS_OCC=1 b --n 15 --N 500000 --censor 0.3 --steps 30 > $O/cfg5_occ1_$r.json 2>>$O/err.txt &&
  b --n 10 --N 1000000 --censor 0.3 --steps 20 > $O/n10c_def_$r.json 2>>$O/err.txt &&
  PHT_CENS_OCC=1 b --n 10 --N 1000000 --censor 0.3 --steps 20 > $O/n10c_occ1_$r.json 2>>$O/err.txt && echo round $r || exit 1
done
python3 - $O <<'PY'
import json, glob, os, sys
for f in sorted(glob.glob(os.path.join(sys.argv[1], "*.json"))):
    d = json.load(open(f)); print(os.path.basename(f), round(d["value"], 1), round(d["ms_per_step"], 4), round(d["roofline"]["kernel_ms"], 4))
PY
