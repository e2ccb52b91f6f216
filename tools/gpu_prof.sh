# rocprofv3 kernel trace + stats of the default bench (4 timed graph replays), then the per-kernel table
set -o pipefail
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; mkdir -p gpurun_out
T=${1:-prof}
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${T}_prof -o ${T} -- python3 bench.py --steps 4 --warmup 2 --no-cpu-baseline --no-census > gpurun_out/${T}_prof.log 2>&1 || exit 14
tail -1 gpurun_out/${T}_prof.log | cut -c1-200
python3 tools/trace_gaps.py gpurun_out/${T}_prof/${T}_kernel_trace.csv --queues > gpurun_out/${T}_queues.txt; tail -40 gpurun_out/${T}_queues.txt
python3 tools/trace_top.py gpurun_out/${T}_prof/${T}_kernel_trace.csv 3 45 > gpurun_out/${T}_top.txt
