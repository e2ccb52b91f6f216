set -o pipefail
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; mkdir -p gpurun_out
T=${1:-r03n}
bash tools/ab_switches.sh ${T} "DFM_SIDE_FROM=0" "DFM_SIDE_FROM=1" "DFM_ATTN_BWD_SIDE_FROM=1" "DFM_SIDE_FROM=1 DFM_ATTN_BWD_SIDE_FROM=1" "DFM_SIDE_FROM=2" "DFM_SIDE_FROM=0" || exit 14
