#!/bin/bash
# host gap A/B: bench.py with the committed library (head.so) against the working tree (OpenBLAS on the
# calling thread for the per-sweep eigensystem), alternating, cfg4 and cfg3
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r05q
mkdir -p $O
cd $GRAFT_REPO_ROOT
H=phasetype_amd/_variants/head.so; N=phasetype_amd/_lib/libPhaseType.so
for r in 1 2 3; do
  PHT_LIB=$H timeout -k 10 200 python3 bench.py --no-cpu-baseline --steps 50 > $O/cfg4_head_$r.json 2>$O/err.txt &&
  PHT_LIB=$N timeout -k 10 200 python3 bench.py --no-cpu-baseline --steps 50 > $O/cfg4_new_$r.json 2>>$O/err.txt &&
  PHT_LIB=$H timeout -k 10 200 python3 bench.py --no-cpu-baseline --n 20 --N 100000 --steps 50 > $O/cfg3_head_$r.json 2>>$O/err.txt &&
  PHT_LIB=$N timeout -k 10 200 python3 bench.py --no-cpu-baseline --n 20 --N 100000 --steps 50 > $O/cfg3_new_$r.json 2>>$O/err.txt &&
  echo round $r || exit 1
done
python3 - $O <<'PY'
import json, glob, os, sys
for f in sorted(glob.glob(os.path.join(sys.argv[1], "cfg*.json"))):
    d = json.load(open(f)); print(os.path.basename(f), round(d["value"], 1), round(d["ms_per_step"], 4), round(d["roofline"]["kernel_ms"], 4))
PY
