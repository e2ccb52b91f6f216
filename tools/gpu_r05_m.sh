# round 5: fused ConvFFN parity + per-stage timing + per-kernel stats at stage 0 / 2
set -o pipefail
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; mkdir -p gpurun_out
T=${1:-r05m}
timeout -k 10 300 python -u -m pytest tests/test_convffn_gpu.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/${T}_convffn.log 2>&1 || { tail -20 gpurun_out/${T}_convffn.log; exit 11; }
tail -1 gpurun_out/${T}_convffn.log
timeout -k 10 300 python -u tools/ffn_kernels_bench.py 0 1 2 > gpurun_out/${T}_ffn.log 2>&1 || exit 12
grep -E "unfused" gpurun_out/${T}_ffn.log
for st in 0; do
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${T}_kt$st -o kt -- python3 tools/ffn_one.py $st mlp 5 > gpurun_out/${T}_kt$st.log 2>&1 || exit 15
echo "stage $st:"; head -9 gpurun_out/${T}_kt$st/kt_kernel_stats.csv | cut -d, -f1-4 | cut -c1-120
done
