# ring-depth switch: GEMM parity with DFM_GLDS_NS=3, then A/B on the bench
set -o pipefail
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; mkdir -p gpurun_out
T=${1:-ns}
DFM_GLDS_NS=3 timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_kernels_gpu.py -k "gemm or group" > gpurun_out/${T}_pytest.log 2>&1 || { tail -30 gpurun_out/${T}_pytest.log; exit 10; }
tail -1 gpurun_out/${T}_pytest.log
bash tools/gpu_r05_ab.sh $T DFM_GLDS_NS 2 3
