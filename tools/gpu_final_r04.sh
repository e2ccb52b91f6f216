# round-4 record: GPU suite, smoke, default bench line + step table, rocprofv3 kernel trace / stats of
# the bench, PMC passes over the measured-dominant kernel (-> profiles/r04_pmc_dominant.json, which
# bench.py reads for roofline.traffic), then configs 2 and 5
set -o pipefail
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; mkdir -p gpurun_out
T=${1:-r04f}
timeout -k 10 900 python -u -m pytest tests -v -m gpu --timeout 180 --timeout-method thread -p no:cacheprovider > gpurun_out/${T}_pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; grep -E "^(FAILED|ERROR)|passed|failed" gpurun_out/${T}_pytest_gpu.log | tail -5
[ $rc -eq 0 ] || exit 11
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${T}_smoke.log 2>&1 || exit 12
tail -1 gpurun_out/${T}_smoke.log
timeout -k 10 400 python -u bench.py --table-out gpurun_out/${T}_step_table.json > gpurun_out/${T}_bench.log 2>&1 || exit 13
tail -1 gpurun_out/${T}_bench.log | cut -c1-300
bash tools/gpu_pmc.sh ${T} gpurun_out/${T}_step_table.json || exit 14
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${T}_stats -o ${T} -- python3 bench.py --no-cpu-baseline > gpurun_out/${T}_stats.log 2>&1 || exit 15
tail -1 gpurun_out/${T}_stats.log | cut -c1-200
rm -f gpurun_out/${T}_stats/${T}_kernel_trace.csv
bash tools/gpu_prof.sh ${T} || exit 16
rm -f gpurun_out/${T}_prof/${T}_kernel_trace.csv
bash tools/gpu_configs.sh ${T} || exit 17
