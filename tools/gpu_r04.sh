# round 4: full GPU suite + smoke + default bench line; optional trailing diagnostic
set -o pipefail
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; mkdir -p gpurun_out
T=${1:-r04}
timeout -k 10 900 python -u -m pytest tests -v -m gpu --timeout 180 --timeout-method thread -p no:cacheprovider > gpurun_out/${T}_pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; grep -E "^(FAILED|ERROR)|passed|failed" gpurun_out/${T}_pytest_gpu.log | tail -12
[ $rc -le 1 ] || exit 11
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${T}_smoke.log 2>&1 || exit 12
tail -1 gpurun_out/${T}_smoke.log
timeout -k 10 400 python -u bench.py --table-out gpurun_out/${T}_step_table.json > gpurun_out/${T}_bench.log 2>&1 || exit 13
tail -1 gpurun_out/${T}_bench.log | cut -c1-600
if [ "$2" = "diag" ]; then timeout -k 10 120 python -u tools/nmf_gx_diag.py > gpurun_out/${T}_nmf_diag.log 2>&1; echo "diag rc=$?"; cat gpurun_out/${T}_nmf_diag.log | tail -5; fi
exit $rc
