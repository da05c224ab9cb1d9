#!/bin/bash
# conflict-free exp table (-D PHT_EXP16: 16 lane-position copies) against HEAD at cfg5 ECS and cfg3 (n = 10's
# exact kernel goes to 258 VGPRs = one wave per SIMD with it, so cfg4 is not a candidate); draws checked identical
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/${TAG:-r05ai}
mkdir -p $O
cd $GRAFT_REPO_ROOT
H=phasetype_amd/_variants/head.so; E=phasetype_amd/_variants/e16.so
timeout -k 10 300 python3 tools/ab.py --libs $H $E --rounds 5 --sweeps 10 --n 15 --N 500000 --censor 0.3 > $O/cfg5.json && echo cfg5 &&
timeout -k 10 300 python3 tools/ab.py --libs $H $E --rounds 5 --sweeps 20 --n 20 --N 100000 > $O/cfg3.json && echo cfg3 &&
timeout -k 10 300 python3 tools/ab.py --libs $H $E --rounds 5 --sweeps 10 --n 15 --N 500000 > $O/n15_exact.json && echo n15
