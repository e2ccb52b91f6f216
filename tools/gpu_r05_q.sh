# round 5: Block C entry points, fused ConvFFN, fp16 ring GEMM (GEMM / fp16 tests), bench + configs 2 / 5
set -o pipefail
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; mkdir -p gpurun_out
T=${1:-r05q}
timeout -k 10 600 python -u -m pytest tests/test_block_capi_gpu.py tests/test_convffn_gpu.py tests/test_fp16_gpu.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/${T}_t1.log 2>&1 || { tail -30 gpurun_out/${T}_t1.log; exit 11; }
tail -1 gpurun_out/${T}_t1.log
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py -x -q -k "gemm or linear" --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/${T}_t2.log 2>&1 || { tail -30 gpurun_out/${T}_t2.log; exit 12; }
tail -1 gpurun_out/${T}_t2.log
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/${T}_bench.log 2>&1 || { tail -5 gpurun_out/${T}_bench.log; exit 13; }
tail -1 gpurun_out/${T}_bench.log | cut -c1-300
bash tools/gpu_configs.sh ${T} || exit 14
