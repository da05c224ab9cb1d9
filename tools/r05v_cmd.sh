#!/bin/bash
# scheduler-flag variants at cfg3 (n = 20, N = 1e5, ECS), two interleaved A/Bs
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r05v
mkdir -p $O
cd $GRAFT_REPO_ROOT
V=phasetype_amd/_variants
L="$V/head.so $V/trk.so $V/nouc.so $V/bias50.so $V/bias0.so"
timeout -k 10 300 python3 tools/ab.py --libs $L --rounds 5 --sweeps 20 --n 20 --N 100000 > $O/cfg3_a.json && echo a &&
timeout -k 10 300 python3 tools/ab.py --libs $L --rounds 5 --sweeps 20 --n 20 --N 100000 > $O/cfg3_b.json && echo b
