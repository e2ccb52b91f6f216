# two A/Bs in one call
set -o pipefail
cd $GRAFT_REPO_ROOT
bash tools/gpu_r05_ab.sh ${1}dw7 DFM_DW7_VAR 0 1 || exit 11
bash tools/gpu_r05_ab.sh ${1}small DFM_FFN_FWD_SMALL 0 1 || exit 12
