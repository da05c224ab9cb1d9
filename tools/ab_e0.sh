#!/bin/bash
# A/B of the first-sojourn E0 fold (base = previous tree, new = in-tree library), ECS at cfg4,
# the 8-GPU shard (125k), cfg5 ECS and cfg3 ECS; timing only (the device spec changed).
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-e0ab}
mkdir -p $O
cd $GRAFT_REPO_ROOT
B=phasetype_amd/_variants/base.so; N=phasetype_amd/_lib/libPhaseType.so
timeout -k 10 200 python3 tools/ab.py --libs $B $N --no-check --rounds 5 --sweeps 10 > $O/cfg4.json && echo cfg4 &&
timeout -k 10 200 python3 tools/ab.py --libs $B $N --no-check --rounds 5 --sweeps 20 --N 125000 > $O/125k.json && echo 125k &&
timeout -k 10 200 python3 tools/ab.py --libs $B $N --no-check --rounds 5 --sweeps 10 --n 15 --N 500000 --censor 0.3 > $O/cfg5.json && echo cfg5 &&
timeout -k 10 200 python3 tools/ab.py --libs $B $N --no-check --rounds 5 --sweeps 20 --n 20 --N 100000 > $O/cfg3.json && echo cfg3
