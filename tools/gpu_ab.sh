# GEMM-routing A/B on one box: GEMM kernel tests first (stop on failure), then the default bench line
# with its census table, then the same step with the named env switch (e.g. DFM_GEMM_RING=0)
set -o pipefail
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; mkdir -p gpurun_out
T=${1:-ab}; SW=${2:-DFM_GEMM_RING=0}
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -v -m gpu -k "gemm or bmm" --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/${T}_pytest_gemm.log 2>&1; rc=$?
echo "gemm tests rc=$rc"; grep -E "^(FAILED|ERROR)|passed|failed" gpurun_out/${T}_pytest_gemm.log | tail -12
[ $rc -eq 0 ] || exit 11
timeout -k 10 300 python -u bench.py --no-cpu-baseline --table-out gpurun_out/${T}_step_table.json > gpurun_out/${T}_bench.log 2>&1 || exit 13
tail -1 gpurun_out/${T}_bench.log | cut -c1-200
env $SW timeout -k 10 300 python -u bench.py --no-cpu-baseline --table-out gpurun_out/${T}_step_table_alt.json > gpurun_out/${T}_bench_alt.log 2>&1 || exit 14
echo "alt ($SW):"; tail -1 gpurun_out/${T}_bench_alt.log | cut -c1-200
timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/${T}_bench2.log 2>&1 || exit 15
echo "default again:"; tail -1 gpurun_out/${T}_bench2.log | cut -c1-200
