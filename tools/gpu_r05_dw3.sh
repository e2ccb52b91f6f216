# streaming 3x3 depthwise: parity tests of the in-tree build, then A/B against a variant build
#   bash tools/gpu_r05_dw3.sh TAG VARIANT_SO
set -o pipefail
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; mkdir -p gpurun_out
T=${1:-dw3}
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_kernels_gpu.py tests/test_convffn_gpu.py tests/test_block_gpu.py > gpurun_out/${T}_pytest.log 2>&1 \
  || { tail -30 gpurun_out/${T}_pytest.log; exit 10; }
tail -2 gpurun_out/${T}_pytest.log
bash tools/gpu_r05_lib_ab.sh $T $2
