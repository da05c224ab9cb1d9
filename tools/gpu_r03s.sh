set -o pipefail
# resident ECS with the warm-start eigensystem: resident GPU tests, then host vs resident at cfg1-3
O=$GRAFT_REPO_ROOT/gpurun_out/r03s; mkdir -p $O; cd $GRAFT_REPO_ROOT
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_resident.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 600 python3 tools/resident_bench.py cfg1 cfg2 cfg3 ECS DCS > $O/resident.jsonl 2> $O/resident.err || { tail -20 $O/resident.err; exit 1; }
python3 -c "
import json
for l in open('$O/resident.jsonl'):
    d=json.loads(l); print(d['config'], d['method'], d['mode'], round(d['sweeps_per_s'],1), round(d['ms_per_step'],4), d['ok'])
"
