set -o pipefail
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; mkdir -p gpurun_out
T=${1:-glds3}
DFM_GLDS_DGRAD_K=128 timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_block_gpu.py -x -q -m gpu -k "gemm or linear or block" --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/${T}_k.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -1 gpurun_out/${T}_k.log
[ $rc -le 1 ] || exit 11
bash tools/ab_switches.sh ${T} "DFM_GLDS_DGRAD_K=640" "DFM_GLDS_DGRAD_K=256" "DFM_GLDS_DGRAD_K=128" "DFM_GLDS_DGRAD_K=640" "DFM_GLDS_DGRAD_K=256" "DFM_GLDS_DGRAD_K=128" || exit 14
