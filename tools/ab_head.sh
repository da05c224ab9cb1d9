#!/bin/bash
# A/B: the committed tree (_variants/head.so, tools/build_variant.py head --ref HEAD) against the
# working tree's library at cfg4 / the 8-GPU shard (125k) / cfg5 ECS / cfg3 ECS, draws checked identical.
# usage (GPU box): tools/ab_head.sh <tag> [--no-check]
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-abhead}
X=${2:-}
mkdir -p $O
cd $GRAFT_REPO_ROOT
H=phasetype_amd/_variants/head.so; N=phasetype_amd/_lib/libPhaseType.so
timeout -k 10 200 python3 tools/ab.py --libs $H $N $X --rounds 5 --sweeps 10 > $O/cfg4.json && echo cfg4 &&
timeout -k 10 200 python3 tools/ab.py --libs $H $N $X --rounds 5 --sweeps 20 --N 125000 > $O/125k.json && echo 125k &&
timeout -k 10 200 python3 tools/ab.py --libs $H $N $X --rounds 5 --sweeps 10 --n 15 --N 500000 --censor 0.3 > $O/cfg5.json && echo cfg5 &&
timeout -k 10 200 python3 tools/ab.py --libs $H $N $X --rounds 5 --sweeps 20 --n 20 --N 100000 > $O/cfg3.json && echo cfg3
