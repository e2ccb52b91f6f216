# full GPU suite + smoke, then the default bench line (reads profiles/r03_pmc_dominant.json)
set -o pipefail
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; mkdir -p gpurun_out
T=${1:-final}
bash tools/gpu_tests.sh ${T} || exit 11
timeout -k 10 400 python -u bench.py --table-out gpurun_out/${T}_step_table.json > gpurun_out/${T}_bench.log 2>&1 || exit 13
tail -1 gpurun_out/${T}_bench.log | cut -c1-400
