# full GPU test suite (+ smoke), stopping the call on any abort / timeout
set -o pipefail
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; mkdir -p gpurun_out
T=${1:-gt}
timeout -k 10 600 python -u -m pytest tests -q -m gpu --timeout 180 --timeout-method thread -p no:cacheprovider > gpurun_out/${T}_pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; grep -E "^(FAILED|ERROR)|passed|failed" gpurun_out/${T}_pytest_gpu.log | tail -8
[ $rc -le 1 ] || exit 11
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${T}_smoke.log 2>&1 || exit 12
tail -1 gpurun_out/${T}_smoke.log
[ $rc -eq 0 ] || exit 1
