set -o pipefail
# PC sampling of the cfg4 ECS sweep (host-trap, time-based), for hot-spot attribution
O=$GRAFT_REPO_ROOT/gpurun_out/pcs; mkdir -p $O; cd /tmp && export TMPDIR=/tmp
timeout -k 10 60 rocprofv3 -L > $O/list.txt 2>&1 || true
grep -i -A3 "pc_sampl\|PC sampl" $O/list.txt | head -40
timeout -k 10 240 rocprofv3 --pc-sampling-beta-enabled --pc-sampling-method ${M:-host_trap} --pc-sampling-unit ${U:-time} --pc-sampling-interval ${I:-1} --output-format csv -d $O/run -o run -- python3 $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline --no-alt --steps 20 > $O/bench.json 2> $O/err.txt || { tail -20 $O/err.txt; exit 1; }
find $O/run -type f | head; 
