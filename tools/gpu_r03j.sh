# GEMM barrier change: GEMM kernel tests, full suite, A/B of GEMM switches
set -o pipefail
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; mkdir -p gpurun_out
T=${1:-r03j}
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q -m gpu -k "gemm or linear" --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/${T}_k.log 2>&1; rc=$?
echo "gemm tests rc=$rc"; grep -E "^E  |passed|failed" gpurun_out/${T}_k.log | head -20
[ $rc -eq 0 ] || exit 11
bash tools/gpu_tests.sh ${T} || exit 12
bash tools/ab_switches.sh ${T} "DFM_GEMM_STREAM=1" "DFM_GEMM_STREAM=2" "DFM_GEMM_WG=3" "DFM_GEMM_STREAM=1" || exit 14
