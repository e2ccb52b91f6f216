set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 500 python -m pytest tests -q -m gpu > gpurun_out/r01_pytest_gpu.log 2>&1 || exit 11
timeout -k 10 400 python bench.py > gpurun_out/r01_bench.log 2>&1 || exit 12
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r01_prof -o r01 -- python3 bench.py --steps 4 --warmup 2 --no-cpu-baseline > gpurun_out/r01_prof.log 2>&1 || exit 13
timeout -k 10 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/r01_pmc_fetch -o f -- python3 tools/dominant_kernel.py > gpurun_out/r01_pmc_fetch.log 2>&1 || exit 14
timeout -k 10 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/r01_pmc_write -o w -- python3 tools/dominant_kernel.py > gpurun_out/r01_pmc_write.log 2>&1 || exit 15
