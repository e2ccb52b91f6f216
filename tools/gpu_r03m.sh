# grouped weight gradients on a side stream / block target: tests with the stream, A/B
set -o pipefail
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; mkdir -p gpurun_out
T=${1:-r03m}
DFM_WGRAD_GROUP_STREAM=1 timeout -k 10 300 python -u -m pytest tests/test_graph_gpu.py tests/test_dp_gpu.py tests/test_segmentor_gpu.py -x -q -m gpu --timeout 180 --timeout-method thread -p no:cacheprovider > gpurun_out/${T}_s.log 2>&1; rc=$?
echo "group-stream tests rc=$rc"; tail -2 gpurun_out/${T}_s.log
[ $rc -le 1 ] || exit 13
bash tools/ab_switches.sh ${T} "DFM_WGRAD_GROUP_STREAM=0" "DFM_WGRAD_GROUP_STREAM=1" "DFM_WG_BLOCKS=1024" "DFM_WG_BLOCKS=256" "DFM_WGRAD_GROUP_STREAM=1 DFM_WG_BLOCKS=1024" "DFM_WGRAD_GROUP_STREAM=0" || exit 14
