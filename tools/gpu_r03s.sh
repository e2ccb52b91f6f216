set -o pipefail
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; mkdir -p gpurun_out
T=${1:-r03s}
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q -m gpu -k "wgrad_group" --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/${T}_k.log 2>&1; rc=$?
echo "group tests rc=$rc"; tail -1 gpurun_out/${T}_k.log
[ $rc -eq 0 ] || exit 11
bash tools/ab_switches.sh ${T} "DFM_WG_BLOCKS=512" "DFM_WG_BLOCKS=1024" "DFM_WGRAD_GROUP=0" "DFM_WG_BLOCKS=512" || exit 14
