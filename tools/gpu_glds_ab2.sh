set -o pipefail
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; mkdir -p gpurun_out
T=${1:-glds2}
bash tools/ab_switches.sh ${T} "DFM_GLDS_SMALL=0" "DFM_GLDS_SMALL=2048" "DFM_GLDS_SMALL=4096" "DFM_GLDS_SMALL=100000" "DFM_GLDS_SMALL=0" "DFM_GLDS_SMALL=2048" "DFM_GLDS_SMALL=4096" || exit 14
