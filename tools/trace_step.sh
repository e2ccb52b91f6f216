# Usage (on the GPU box via gpurun): bash tools/trace_step.sh TAG [extra bench args]
# Full per-dispatch kernel trace (rocprofv3 --kernel-trace, CSV) of a few bench steps, once eager
# (per-kernel durations in launch order; the depth-branch ConvFFN and attention-backward side streams
# still overlap the main stream, so concurrent kernels share the GPU) and once as the default captured step
# (what the bench times). tools/trace_table.py turns the CSVs into per-shape tables.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=${1:-trace}
shift
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/${T}_eager -o k -- \
  python3 bench.py --steps 3 --warmup 2 --no-cpu-baseline --no-census --eager "$@" > gpurun_out/${T}_eager.log 2>&1 || exit 21
tail -1 gpurun_out/${T}_eager.log | cut -c1-200
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/${T}_graph -o k -- \
  python3 bench.py --steps 3 --warmup 2 --no-cpu-baseline --no-census "$@" > gpurun_out/${T}_graph.log 2>&1 || exit 22
tail -1 gpurun_out/${T}_graph.log | cut -c1-200
echo done
