#!/bin/bash
# A/B: fold (HEAD) vs the tree (Elast live range) at cfg4 / 125k / cfg5; n = 20 one vs two waves (w2) at cfg3 and 5e5
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-s5}
mkdir -p $O
cd $GRAFT_REPO_ROOT
F=phasetype_amd/_variants/fold.so; N=phasetype_amd/_lib/libPhaseType.so; W=phasetype_amd/_variants/w2.so
timeout -k 10 200 python3 tools/ab.py --libs $F $N --rounds 5 --sweeps 10 > $O/cfg4.json && echo cfg4 &&
timeout -k 10 200 python3 tools/ab.py --libs $F $N --rounds 5 --sweeps 20 --N 125000 > $O/125k.json && echo 125k &&
timeout -k 10 200 python3 tools/ab.py --libs $F $N $W --rounds 5 --sweeps 20 --n 20 --N 100000 > $O/cfg3.json && echo cfg3 &&
timeout -k 10 200 python3 tools/ab.py --libs $N $W --rounds 3 --sweeps 10 --n 20 --N 500000 > $O/n20_5e5.json && echo n20 &&
timeout -k 10 200 python3 tools/ab.py --libs $F $N --rounds 5 --sweeps 10 --n 15 --N 500000 --censor 0.3 > $O/cfg5.json && echo cfg5
