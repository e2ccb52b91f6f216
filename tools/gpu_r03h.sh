# new-kernel tests, then the full suite, then A/B of the fused DW backward and the second attention-backward stream
set -o pipefail
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; mkdir -p gpurun_out
T=${1:-r03h}
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q -m gpu -k "fused_bwd or gelu_grad or act3 or dwconv" --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/${T}_k.log 2>&1; rc=$?
echo "kernel tests rc=$rc"; grep -E "^E  |passed|failed" gpurun_out/${T}_k.log | head -20
[ $rc -eq 0 ] || exit 11
bash tools/gpu_tests.sh ${T} || exit 12
DFM_ATTN_BWD_STREAM2=1 timeout -k 10 300 python -u -m pytest tests/test_block_gpu.py tests/test_graph_gpu.py tests/test_segmentor_gpu.py -x -q -m gpu --timeout 180 --timeout-method thread -p no:cacheprovider > gpurun_out/${T}_s2.log 2>&1; rc=$?
echo "stream2 tests rc=$rc"; tail -2 gpurun_out/${T}_s2.log
[ $rc -le 1 ] || exit 13
bash tools/ab_switches.sh ${T} "DFM_DW_FUSED_BWD=1" "DFM_DW_FUSED_BWD=0" "DFM_ATTN_BWD_STREAM2=1" "DFM_DW_FUSED_BWD=1" || exit 14
