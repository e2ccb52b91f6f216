set -o pipefail
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; mkdir -p gpurun_out
T=${1:-r03r}
bash tools/gpu_tests.sh ${T} || exit 12
bash tools/ab_switches.sh ${T} "DFM_FWD_GROUP=0" "DFM_DW_F3=0" "DFM_FWD_GROUP=0" || exit 14
