# A/B of stream / GEMM switches on top of the attention-backward side stream; DP + graph tests
set -o pipefail
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; mkdir -p gpurun_out
T=${1:-r03d}
timeout -k 10 300 python -u -m pytest tests/test_dp_gpu.py -x -q -m gpu --timeout 280 --timeout-method thread -p no:cacheprovider > gpurun_out/${T}_dp.log 2>&1; rc=$?
echo "dp rc=$rc"; tail -2 gpurun_out/${T}_dp.log
[ $rc -le 1 ] || exit 11
B=DFM_ATTN_BWD_STREAM=1
bash tools/ab_switches.sh ${T} "$B" "$B DFM_ATTN_STREAM=1" "$B DFM_GEMM_WG=3" "$B DFM_GEMM_WG=4" "$B DFM_WGRAD_STREAM=1" "$B DFM_DW_F7=1" "$B DFM_DW_F7=2" "$B" || exit 13
echo done
