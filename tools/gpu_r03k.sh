set -o pipefail
# kernel trace of the resident update kernel (device eigensystem) at n = 3, 10, 20
O=$GRAFT_REPO_ROOT/gpurun_out/r03k; mkdir -p $O; cd /tmp && export TMPDIR=/tmp
for n in 3 10 20; do
  timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/n$n -o run -- python3 $GRAFT_REPO_ROOT/tools/prof_resident.py $n 2000 ECS 200 > $O/n$n.out 2> $O/n$n.err || { tail $O/n$n.err; exit 1; }
  cat $O/n$n.out; head -6 $O/n$n/run_kernel_stats.csv | cut -d, -f1-4
done
