set -o pipefail
# resident chain with the device eigensystem (ECS/DCS): GPU tests, then the host-vs-resident bench
O=$GRAFT_REPO_ROOT/gpurun_out/r03j; mkdir -p $O; cd $GRAFT_REPO_ROOT
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_resident.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
grep -E "passed|failed" $O/pytest.log | tail -3
timeout -k 10 900 python3 tools/resident_bench.py > $O/resident.jsonl 2> $O/resident.err || { tail -20 $O/resident.err; exit 1; }
python3 -c "
import json
for l in open('$O/resident.jsonl'):
    d=json.loads(l); print(d['config'], d['method'], d['mode'], round(d['sweeps_per_s'],1), round(d['ms_per_step'],4), d['ok'])
"
