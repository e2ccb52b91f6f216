set -o pipefail
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -q -m gpu -x --timeout 180 --timeout-method thread -p no:cacheprovider > gpurun_out/r03a_pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -15 gpurun_out/r03a_pytest_gpu.log
if [ $rc -gt 1 ]; then exit 11; fi
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r03a_smoke.log 2>&1 || exit 12
tail -1 gpurun_out/r03a_smoke.log
timeout -k 10 400 python -u bench.py --table-out gpurun_out/r03a_step_table.json > gpurun_out/r03a_bench.log 2>&1 || exit 13
tail -1 gpurun_out/r03a_bench.log | cut -c1-600
