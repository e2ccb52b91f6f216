# Usage (GPU box): bash tools/gpu_pmc_kernels.sh TAG STEP_TABLE_JSON SUBSTR...
# HBM traffic (FETCH_SIZE x2 + WRITE_SIZE) and MFMA busy of chosen census kernels over bench.py's
# eager steps: one rocprofv3 pass per counter group for all of them (kernel-include regex =
# the substrings' alternation), then tools/pmc_dominant.py per kernel -> gpurun_out/TAG_<i>.json
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=$1; TABLE=$2; shift 2
mkdir -p gpurun_out
RE=$(python3 -c "import re,sys; print('|'.join(re.escape(s) for s in sys.argv[1:]))" "$@")
echo "kernel regex: $RE"
BENCH="bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-census --eager"
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "$RE" --output-format csv -d gpurun_out/${T}_fetch -o f -- python3 $BENCH > gpurun_out/${T}_fetch.log 2>&1 || exit 21
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "$RE" --output-format csv -d gpurun_out/${T}_write -o w -- python3 $BENCH > gpurun_out/${T}_write.log 2>&1 || exit 22
timeout -s KILL 300 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-include-regex "$RE" --output-format csv -d gpurun_out/${T}_mfma -o m -- python3 $BENCH > gpurun_out/${T}_mfma.log 2>&1 || exit 23
i=0
for s in "$@"; do
  i=$((i+1))
  python3 tools/pmc_dominant.py $TABLE gpurun_out/${T}_fetch gpurun_out/${T}_write gpurun_out/${T}_mfma gpurun_out/${T}_$i.json "$s" || exit 24
done
