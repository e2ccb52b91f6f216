# weight-gradient ring route: parity with DFM_WGRAD_RING=1, then A/B against the register route
set -o pipefail
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; mkdir -p gpurun_out
T=${1:-wgring}
DFM_WGRAD_RING=1 timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_kernels_gpu.py -k "wgrad or gemm" > gpurun_out/${T}_pytest_k.log 2>&1 || { tail -30 gpurun_out/${T}_pytest_k.log; exit 10; }
tail -1 gpurun_out/${T}_pytest_k.log
DFM_WGRAD_RING=1 timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_block_gpu.py tests/test_convffn_gpu.py tests/test_block_capi_gpu.py > gpurun_out/${T}_pytest_b.log 2>&1 || { tail -30 gpurun_out/${T}_pytest_b.log; exit 10; }
tail -1 gpurun_out/${T}_pytest_b.log
bash tools/gpu_r05_ab.sh $T DFM_WGRAD_RING 0 1
