set -o pipefail
# the full GPU test suite (one process), log under gpurun_out/<tag>/
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-full}; mkdir -p $O; cd $GRAFT_REPO_ROOT
timeout -k 10 1100 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu_full.log 2>&1 || { tail -40 $O/pytest_gpu_full.log; exit 1; }
tail -1 $O/pytest_gpu_full.log
