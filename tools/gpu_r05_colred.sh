# colred_vec with y presence at compile time: parity (full suite), step A/B vs the HEAD build
set -o pipefail
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; mkdir -p gpurun_out
T=${1:-colred}
timeout -k 10 700 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > gpurun_out/${T}_pytest.log 2>&1 || { tail -30 gpurun_out/${T}_pytest.log; exit 10; }
tail -1 gpurun_out/${T}_pytest.log
bash tools/gpu_r05_lib_ab.sh $T dformer_amd/variants/lib_base.so
