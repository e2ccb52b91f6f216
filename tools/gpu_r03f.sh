set -o pipefail
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; mkdir -p gpurun_out
T=${1:-r03f}
NCCL_DEBUG=WARN TORCH_NCCL_ASYNC_ERROR_HANDLING=0 timeout -k 10 400 python -u -m pytest tests/test_abi.py tests/test_block_gpu.py tests/test_graph_gpu.py -x -v -s -m gpu --timeout 180 --timeout-method thread -p no:cacheprovider > gpurun_out/${T}.log 2>&1; rc=$?
echo "rc=$rc"; grep -E "forced-collectives failure|PASSED|FAILED|NCCL WARN|Error" gpurun_out/${T}.log | tail -30
