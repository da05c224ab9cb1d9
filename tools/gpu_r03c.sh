set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r03c; mkdir -p $O; cd $GRAFT_REPO_ROOT
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_resident.py -v --timeout 150 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -3 $O/pytest.log; grep -E "FAILED|ERROR|Error" $O/pytest.log | head -20
[ $rc -le 1 ] || exit $rc
timeout -k 10 400 python3 tools/resident_bench.py > $O/resident.jsonl 2> $O/resident.err || { tail $O/resident.err; exit 1; }
python3 -c "
import json
for l in open('$O/resident.jsonl'):
    d=json.loads(l); print(d['config'], d['method'], d['mode'], round(d['sweeps_per_s'],1), 'ms', round(d['ms_per_step'],4), 'kern', round(d['kernel_ms_per_step'],4), d['ok'])"
