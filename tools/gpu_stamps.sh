#!/bin/bash
# Per-phase cycle stamps of the ECS kernel (PHT_STAMPS variant build) at the
# lone-wave (top64), strong-scaling (125k) and single-GPU (1e6) shard sizes.
# usage (GPU box): tools/gpu_stamps.sh <tag> <variant.so>
set -o pipefail
TAG=$1; LIB=$2
O=$GRAFT_REPO_ROOT/gpurun_out/stamps_$TAG
mkdir -p $O
cd $GRAFT_REPO_ROOT
PHT_LIB=$LIB timeout -k 10 120 python3 tools/stamps.py --top 64 > $O/top64.json 2>&1 &&
PHT_LIB=$LIB timeout -k 10 120 python3 tools/stamps.py --N 125000 > $O/125k.json 2>&1 &&
PHT_LIB=$LIB timeout -k 10 120 python3 tools/stamps.py > $O/1M.json 2>&1
