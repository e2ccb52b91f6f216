# round 5: fused ConvFFN A/B (backward occupancy variant) + SQ counters of the fused kernels at stage 0
set -o pipefail
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; mkdir -p gpurun_out
T=${1:-r05e}
timeout -k 10 300 python -u -m pytest tests/test_convffn_gpu.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/${T}_convffn.log 2>&1 || { tail -20 gpurun_out/${T}_convffn.log; exit 11; }
tail -1 gpurun_out/${T}_convffn.log
timeout -k 10 300 python -u tools/ffn_kernels_bench.py 0 1 > gpurun_out/${T}_ffn.log 2>&1 || exit 12
grep -E "unfused" gpurun_out/${T}_ffn.log
bash tools/ffn_pmc.sh ${T}pmc 0 mlp || exit 14
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${T}_kt -o kt -- python3 tools/ffn_one.py 0 mlp 5 > gpurun_out/${T}_kt.log 2>&1 || exit 15
echo done
