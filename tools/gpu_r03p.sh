set -o pipefail
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; mkdir -p gpurun_out
T=${1:-r03p}
DFM_GEMM_STREAM=3 DFM_GEMM_SK64=1 timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_block_gpu.py -x -q -m gpu -k "gemm or linear or block" --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/${T}_k.log 2>&1; rc=$?
echo "knob tests rc=$rc"; tail -1 gpurun_out/${T}_k.log
[ $rc -le 1 ] || exit 11
bash tools/ab_switches.sh ${T} "DFM_GEMM_STREAM=1" "DFM_GEMM_STREAM=3" "DFM_GEMM_SK64=1" "DFM_GEMM_STREAM=3 DFM_GEMM_SK64=1" "DFM_GEMM_STREAM=1" || exit 14
