# grouped weight gradients: kernel test, full suite, A/B
set -o pipefail
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; mkdir -p gpurun_out
T=${1:-r03k}
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q -m gpu -k "wgrad_group or gemm" --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/${T}_k.log 2>&1; rc=$?
echo "group tests rc=$rc"; grep -E "^E  |passed|failed" gpurun_out/${T}_k.log | head -20
[ $rc -eq 0 ] || exit 11
bash tools/gpu_tests.sh ${T} || exit 12
bash tools/ab_switches.sh ${T} "DFM_WGRAD_GROUP=1" "DFM_WGRAD_GROUP=0" "DFM_WGRAD_GROUP=1" || exit 14
