# round 5: deferred split-K combines — parity of the Block / end-to-end / kernel tests, then step A/B
set -o pipefail
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; mkdir -p gpurun_out
T=${1:-r05t}
timeout -k 10 900 python -u -m pytest tests/test_block_gpu.py tests/test_segmentor_gpu.py tests/test_fp16_gpu.py tests/test_graph_gpu.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/${T}_t.log 2>&1 || { tail -30 gpurun_out/${T}_t.log; exit 11; }
tail -1 gpurun_out/${T}_t.log
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py -x -q -k "group or wgrad or partial or deferred" --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/${T}_tk.log 2>&1 || { tail -30 gpurun_out/${T}_tk.log; exit 12; }
tail -1 gpurun_out/${T}_tk.log
bash tools/gpu_r05_ab.sh ${T}ab DFM_DEFER_COMBINE 0 1 || exit 13
