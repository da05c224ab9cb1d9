set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r03d; mkdir -p $O; cd $GRAFT_REPO_ROOT
timeout -k 10 900 python3 -u -m pytest tests -m gpu -v --timeout 150 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -3 $O/pytest.log; grep -E "FAILED|ERROR|Error" $O/pytest.log | head -20
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 python3 tools/chains.py > $O/chains.jsonl 2> $O/chains.err; tail -20 $O/chains.jsonl
exit $rc
