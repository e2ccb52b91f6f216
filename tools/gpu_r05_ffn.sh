# round 5: fused ConvFFN parity tests + isolated timing (unfused chain vs fused entry points) + rocprof stats
set -o pipefail
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; mkdir -p gpurun_out
T=${1:-r05b}
timeout -k 10 600 python -u -m pytest tests/test_convffn_gpu.py -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/${T}_convffn.log 2>&1; rc=$?
echo "convffn pytest rc=$rc"; grep -E "PASSED|FAILED|ERROR|passed|failed|Error|assert" gpurun_out/${T}_convffn.log | tail -30
[ $rc -eq 0 ] || exit 11
timeout -k 10 300 python -u tools/ffn_kernels_bench.py 0 1 2 > gpurun_out/${T}_ffn.log 2>&1 || exit 12
grep -E "unfused|FUSED" gpurun_out/${T}_ffn.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_prof -o k -- python3 tools/ffn_kernels_bench.py 0 1 2 > gpurun_out/${T}_prof.log 2>&1 || exit 13
echo done
