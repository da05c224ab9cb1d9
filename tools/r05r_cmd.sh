#!/bin/bash
# MHRS cfg4: lane utilisation / tail share per search round (diag build), and a kernel trace of the
# bench's fresh-chain window (per-kernel durations and the gaps between launches)
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r05r
mkdir -p $O
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
PHT_LIB=phasetype_amd/_variants/mdiag.so timeout -k 10 200 python3 tools/mhrs_diag.py > $O/diag_cfg4.jsonl 2>$O/diag.err && echo diag &&
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $O/trace -o run -- python3 bench.py --method MHRS --steps 30 --no-cpu-baseline --no-alt > $O/bench.json 2>$O/bench.err && echo trace
