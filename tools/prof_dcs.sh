#!/bin/bash
# PMC passes over a DCS bench (cfg5-shaped): instruction mix, lane
# utilisation, waits.  usage (GPU box): tools/prof_dcs.sh <tag> [n] [extra env, e.g. PHT_DCS_LEGACY=1]
set -o pipefail
TAG=${1:-dcs}
NS=${2:-15}
O=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
i=0
while read -r GROUP; do
  [ -z "$GROUP" ] && continue
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $GROUP --output-format csv -d $O/p$i -o run -- \
    python3 $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline --n $NS --N 500000 --censor 0.3 --method DCS --steps 2 --warmup 1 > $O/p$i.json 2> $O/p$i.err || exit $?
done <<'GROUPS'
SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU
SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_INSTS_BRANCH SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU_FLOPS_FP64 SQ_THREAD_CYCLES_VALU
GROUPS
cd $GRAFT_REPO_ROOT && python3 tools/pmc_summary.py $O $O/summary.json > /dev/null && echo ok
