# focused: the graph/collective tests with the attention-backward side stream, then the 2-rank DP test
set -o pipefail
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; mkdir -p gpurun_out
T=${1:-r03c}
DFM_ATTN_BWD_STREAM=1 timeout -k 10 300 python -u -m pytest tests/test_graph_gpu.py -x -v -s -m gpu --timeout 180 --timeout-method thread -p no:cacheprovider > gpurun_out/${T}_graph.log 2>&1; rc=$?
echo "graph rc=$rc"; grep -E "PASS|FAIL|Error|assert" gpurun_out/${T}_graph.log | head -20
[ $rc -le 1 ] || exit 11
timeout -k 10 300 python -u -m pytest tests/test_dp_gpu.py -x -v -m gpu --timeout 280 --timeout-method thread -p no:cacheprovider > gpurun_out/${T}_dp.log 2>&1; rc=$?
echo "dp rc=$rc"; tail -3 gpurun_out/${T}_dp.log
