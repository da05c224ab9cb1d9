#!/bin/bash
# PfCum (precomputed running sums of the Pf categorical scan): parity files, then A/B against HEAD
# (head.so) for MHRS cfg4 / cfg5, ECS cfg5 (censored scan) and UNIF cfg4; draws checked identical
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/${TAG:-r05ac}
mkdir -p $O
cd $GRAFT_REPO_ROOT
H=phasetype_amd/_variants/head.so; N=phasetype_amd/_lib/libPhaseType.so
timeout -k 10 500 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_edges.py tests/test_gpu_bridge.py > $O/tests.txt 2>&1 && echo tests ok || { tail -30 $O/tests.txt; exit 1; }
timeout -k 10 300 python3 tools/ab.py --libs $H $N --method MHRS --rounds 5 --sweeps 10 > $O/mhrs_cfg4.json && echo mhrs4 &&
timeout -k 10 300 python3 tools/ab.py --libs $H $N --method MHRS --rounds 5 --sweeps 10 --n 15 --N 500000 --censor 0.3 > $O/mhrs_cfg5.json && echo mhrs5 &&
timeout -k 10 300 python3 tools/ab.py --libs $H $N --rounds 5 --sweeps 10 --n 15 --N 500000 --censor 0.3 > $O/ecs_cfg5.json && echo ecs5 &&
timeout -k 10 300 python3 tools/ab.py --libs $H $N --method UNIF --rounds 5 --sweeps 20 > $O/unif_cfg4.json && echo unif4
