#!/bin/bash
# PMC passes over bench.py (one rocprofv3 run per counter group; counters
# only with --kernel-trace, as the pool requires).  Run on the GPU box.
# usage: tools/prof_pmc.sh <tag> [bench args...]
set -o pipefail
TAG=$1; shift
OUT=$GRAFT_REPO_ROOT/gpurun_out/pmc_$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
i=0
while read -r GROUP; do
  [ -z "$GROUP" ] && continue
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc $GROUP --output-format csv -d $OUT/p$i -o run -- \
    python3 $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline --no-alt "$@" > $OUT/p$i.bench.json 2> $OUT/p$i.err || exit $?
  echo "pass $i done: $GROUP"
done <<'GROUPS'
SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VALU_FLOPS_FP64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_SALU
SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS
FETCH_SIZE
WRITE_SIZE
SQ_INSTS_FLAT SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE
GROUPS
