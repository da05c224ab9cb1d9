#!/bin/bash
# scheduler-flag variants (tools/build_variant.py --flag=-mllvm --flag=...) against HEAD, ECS cfg4 / cfg5 / 125k
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/${TAG:-r05t}
mkdir -p $O
cd $GRAFT_REPO_ROOT
V=phasetype_amd/_variants
L="$V/head.so $V/nouc.so $V/bias0.so $V/nb0.so"
timeout -k 10 300 python3 tools/ab.py --libs $L --rounds 5 --sweeps 10 > $O/cfg4.json && echo cfg4 &&
timeout -k 10 300 python3 tools/ab.py --libs $L --rounds 5 --sweeps 10 --n 15 --N 500000 --censor 0.3 > $O/cfg5.json && echo cfg5 &&
timeout -k 10 300 python3 tools/ab.py --libs $L --rounds 5 --sweeps 20 --N 125000 > $O/125k.json && echo 125k
