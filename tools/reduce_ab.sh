#!/bin/bash
# Statistics all-reduce A/B under torchrun (one rank, RCCL; GPU box): the
# in-library RCCL all-reduce on the sweep stream (default) against the host
# callback through torch.distributed (PHT_STATS_REDUCE=callback), alternating.
# (--states/--obs: torchrun takes --n as an ambiguous prefix of its options)
# usage: tools/reduce_ab.sh <tag>
set -o pipefail
TAG=${1:-reduce}
O=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $O
cd $GRAFT_REPO_ROOT
port=29611
for rep in 1 2; do
  for cfg in "10 1000000 20" "10 125000 100" "5 10000 200"; do
    set -- $cfg
    for mode in rccl callback; do
      port=$((port + 1))
      PHT_STATS_REDUCE=$mode timeout -k 10 180 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 1 \
        --master-addr 127.0.0.1 --master-port $port bench.py --gpus 1 --no-cpu-baseline --no-weak \
        --states $1 --obs $2 --steps $3 --warmup 3 > $O/${mode}_n$1_N$2_$rep.json 2> $O/${mode}_n$1_N$2_$rep.err || exit 1
      python3 -c "import json; a=[json.loads(l) for l in open('$O/${mode}_n$1_N$2_$rep.json') if l.startswith('{')][0]; print('$mode n=$1 N=$2 rep $rep', round(a['ms_per_step'],4), 'ms/step', round(a['roofline']['kernel_ms'],4), 'kernel ms', a['config']['stats_reduce'])"
    done
  done
done
