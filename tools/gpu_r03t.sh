set -o pipefail
# bench.py's multi-rank flow on one GPU: 2 ranks over gloo (host-callback reduce), as the driver's N>1 runs minus RCCL
O=$GRAFT_REPO_ROOT/gpurun_out/r03t; mkdir -p $O; cd $GRAFT_REPO_ROOT
PHT_DIST_BACKEND=gloo timeout -k 10 400 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 10 --warmup 2 > $O/bench2.json 2> $O/bench2.err || { tail -30 $O/bench2.err; exit 1; }
cat $O/bench2.json
