# Usage (on the GPU box via gpurun): bash tools/gpu_round.sh TAG [tests|notests] [bench args...]
# GPU parity tests (all, failures listed), the bench JSON + per-kernel table, rocprofv3 kernel stats.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=${1:-run}
MODE=${2:-tests}
shift 2 2>/dev/null
mkdir -p gpurun_out
if [ "$MODE" = "tests" ]; then
  timeout -k 10 900 python -u -m pytest tests -q -m gpu --timeout 180 --timeout-method thread -p no:cacheprovider > gpurun_out/${T}_pytest_gpu.log 2>&1
  rc=$?
  echo "pytest rc=$rc"; tail -3 gpurun_out/${T}_pytest_gpu.log
  # 0 all passed, 1 some tests failed: go on; anything else (timeout, crash) ends the call here
  if [ $rc -gt 1 ]; then exit 11; fi
fi
timeout -k 10 400 python -u bench.py --table-out gpurun_out/${T}_step_table.json "$@" > gpurun_out/${T}_bench.log 2>&1 || exit 12
tail -1 gpurun_out/${T}_bench.log | cut -c1-600
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${T}_prof -o ${T} -- python3 bench.py --steps 4 --warmup 2 --no-cpu-baseline --no-census "$@" > gpurun_out/${T}_prof.log 2>&1 || exit 13
echo done
