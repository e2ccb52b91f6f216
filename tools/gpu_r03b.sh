# round-3 evidence pass: GPU tests, FFN A/B, fused-FFN switch A/B, rocprofv3 kernel stats of the default bench
set -o pipefail
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; mkdir -p gpurun_out
T=${1:-r03b}
timeout -k 10 600 python -u -m pytest tests -q -m gpu --timeout 180 --timeout-method thread -p no:cacheprovider > gpurun_out/${T}_pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -4 gpurun_out/${T}_pytest_gpu.log
if [ $rc -gt 1 ]; then exit 11; fi
timeout -k 10 300 python -u tools/ffn_ab.py 10 > gpurun_out/${T}_ffn_ab.txt 2>&1 || exit 12
cat gpurun_out/${T}_ffn_ab.txt
DFM_ATTN_BWD_STREAM=1 timeout -k 10 300 python -u -m pytest tests/test_block_gpu.py tests/test_graph_gpu.py tests/test_segmentor_gpu.py -q -m gpu --timeout 180 --timeout-method thread -p no:cacheprovider > gpurun_out/${T}_pytest_attnbwd.log 2>&1; echo "attn-bwd-stream pytest rc=$?"; tail -2 gpurun_out/${T}_pytest_attnbwd.log
bash tools/ab_switches.sh ${T} "DFM_FUSED_FFN=0" "DFM_FUSED_FFN=1" "DFM_ATTN_BWD_STREAM=1" "DFM_ATTN_BWD_STREAM=0" || exit 13
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${T}_prof -o ${T} -- python3 bench.py --steps 4 --warmup 2 --no-cpu-baseline --no-census > gpurun_out/${T}_prof.log 2>&1 || exit 14
echo done
