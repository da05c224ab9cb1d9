#!/bin/bash
# censored ECS kernel at n = 15 with K envelope points in LDS (-D PHT_CENS_K15=K) against HEAD (private envelope), cfg5 ECS, twice
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r05w
mkdir -p $O
cd $GRAFT_REPO_ROOT
V=phasetype_amd/_variants
L="$V/head.so $V/ck5.so $V/ck9.so $V/ck13.so"
timeout -k 10 300 python3 tools/ab.py --libs $L --rounds 5 --sweeps 10 --n 15 --N 500000 --censor 0.3 > $O/cfg5_a.json && echo a &&
timeout -k 10 300 python3 tools/ab.py --libs $L --rounds 5 --sweeps 10 --n 15 --N 500000 --censor 0.3 > $O/cfg5_b.json && echo b
