#!/bin/bash
# uniform-key Philox: parity (bit-exact suites) then A/B against HEAD at the ECS configs and MHRS cfg4/cfg5
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/${TAG:-r05p}
mkdir -p $O
cd $GRAFT_REPO_ROOT
H=phasetype_amd/_variants/head.so; N=phasetype_amd/_lib/libPhaseType.so
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py > $O/parity.txt 2>&1 && echo parity ok &&
tools/ab_head.sh ${TAG:-r05p}/ab &&
timeout -k 10 200 python3 tools/ab.py --libs $H $N --method MHRS --rounds 5 --sweeps 10 > $O/mhrs_cfg4.json && echo mhrs4 &&
timeout -k 10 200 python3 tools/ab.py --libs $H $N --method MHRS --rounds 5 --sweeps 10 --n 15 --N 500000 --censor 0.3 > $O/mhrs_cfg5.json && echo mhrs5
