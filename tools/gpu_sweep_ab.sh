# per-shape GEMM census replay (graph-timed) with the default routing and with an env switch
set -o pipefail
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; mkdir -p gpurun_out
T=${1:-sw}; SW=${2:-DFM_GEMM_RING=0}
timeout -k 10 400 python -u tools/gemm_sweep.py --no-splits --graph --out gpurun_out/${T}_sweep.json > gpurun_out/${T}_sweep.log 2>&1 || exit 11
tail -1 gpurun_out/${T}_sweep.log
env $SW timeout -k 10 400 python -u tools/gemm_sweep.py --no-splits --graph --out gpurun_out/${T}_sweep_alt.json > gpurun_out/${T}_sweep_alt.log 2>&1 || exit 12
tail -1 gpurun_out/${T}_sweep_alt.log
