# Usage (on the GPU box via gpurun): bash tools/gpu_round2.sh TAG [tests|notests]
# GPU parity tests; PMC passes over the dominant kernel (into profiles/r02_dominant_pmc.json so the
# bench line carries its measured traffic); the bench JSON + step table; rocprofv3 kernel stats.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=${1:-run}
mkdir -p gpurun_out
if [ "${2:-tests}" = "tests" ]; then
  timeout -k 10 900 python -u -m pytest tests -q -m gpu --timeout 180 --timeout-method thread -p no:cacheprovider > gpurun_out/${T}_pytest_gpu.log 2>&1
  rc=$?
  echo "pytest rc=$rc"; tail -3 gpurun_out/${T}_pytest_gpu.log
  if [ $rc -gt 1 ]; then exit 11; fi
fi
bash tools/gpu_pmc.sh ${T}p profiles/r02_step_table.json > gpurun_out/${T}_pmc.log 2>&1 || exit 12
cp gpurun_out/${T}p_dominant_pmc.json profiles/r02_dominant_pmc.json
tail -1 gpurun_out/${T}_pmc.log | cut -c1-400
timeout -k 10 400 python -u bench.py --table-out gpurun_out/${T}_step_table.json > gpurun_out/${T}_bench.log 2>&1 || exit 13
tail -1 gpurun_out/${T}_bench.log | cut -c1-300
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${T}_prof -o ${T} -- python3 bench.py --steps 4 --warmup 2 --no-cpu-baseline --no-census > gpurun_out/${T}_prof.log 2>&1 || exit 14
echo done
