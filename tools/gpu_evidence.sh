# Usage (on the GPU box via gpurun): bash tools/gpu_evidence.sh TAG [skip-tests]
# GPU parity tests, bench JSON, rocprofv3 kernel stats of the bench, PMC traffic of the dominant kernel.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=${1:-run}
mkdir -p gpurun_out
if [ "$2" != "skip-tests" ]; then
timeout -k 10 500 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/${T}_pytest_gpu.log 2>&1 || exit 11
fi
timeout -k 10 400 python bench.py > gpurun_out/${T}_bench.log 2>&1 || exit 12
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${T}_prof -o ${T} -- python3 bench.py --steps 4 --warmup 2 --no-cpu-baseline > gpurun_out/${T}_prof.log 2>&1 || exit 13
timeout -k 10 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/${T}_pmc_fetch -o f -- python3 tools/dominant_kernel.py > gpurun_out/${T}_pmc_fetch.log 2>&1 || exit 14
timeout -k 10 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/${T}_pmc_write -o w -- python3 tools/dominant_kernel.py > gpurun_out/${T}_pmc_write.log 2>&1 || exit 15
