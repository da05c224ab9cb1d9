#!/bin/bash
# PMC counters of ONE lone wavefront (the 64 longest paths of the bench data
# set): instructions and cycles per round of the latency floor.
# usage (GPU box): tools/prof_lone.sh <tag>
set -o pipefail
TAG=${1:-lone}
O=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 90 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY --output-format csv -d $O/p1 -o run -- python3 $GRAFT_REPO_ROOT/tools/latency.py --Ns ${SPEC:-top64} --variants g1o2 --sweeps 3 > $O/p1.json 2> $O/p1.err || exit 1
timeout -s KILL 90 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU_FLOPS_FP64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_BRANCH SQ_INSTS_SMEM SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_WAIT_ANY --output-format csv -d $O/p2 -o run -- python3 $GRAFT_REPO_ROOT/tools/latency.py --Ns ${SPEC:-top64} --variants g1o2 --sweeps 3 > $O/p2.json 2> $O/p2.err || exit 1
echo ok
