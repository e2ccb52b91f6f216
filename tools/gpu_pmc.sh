# Usage (on the GPU box via gpurun): bash tools/gpu_pmc.sh TAG STEP_TABLE_JSON [N]
# PMC passes (one counter group per run) over bench.py's eager steps, filtered to the step's N (default 2)
# largest census kernels (the measured-dominant one and its runner-up: the two swap between boxes when
# their census times are close, and bench.py reports both), then tools/pmc_dominant.py per kernel ->
# gpurun_out/TAG_pmc_<i>.json (i = census rank).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=${1:-pmc}
TABLE=${2:-profiles/r05_step_table.json}
N=${3:-2}
mkdir -p gpurun_out
RE=$(python3 -c "
import json, re
t = json.load(open('$TABLE'))
names = list(t['kernels'])[:$N]
print('|'.join(re.escape(re.search(r'(\w+<[^()]*>)\(', n).group(1)) for n in names))")
echo "kernel regex: $RE"
BENCH="bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-census --eager"
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "$RE" --output-format csv -d gpurun_out/${T}_fetch -o f -- python3 $BENCH > gpurun_out/${T}_fetch.log 2>&1 || exit 21
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "$RE" --output-format csv -d gpurun_out/${T}_write -o w -- python3 $BENCH > gpurun_out/${T}_write.log 2>&1 || exit 22
timeout -s KILL 300 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-include-regex "$RE" --output-format csv -d gpurun_out/${T}_mfma -o m -- python3 $BENCH > gpurun_out/${T}_mfma.log 2>&1 || exit 23
for i in $(seq 1 $N); do
  NAME=$(python3 -c "import json; print(list(json.load(open('$TABLE'))['kernels'])[$i - 1])")
  python3 tools/pmc_dominant.py $TABLE gpurun_out/${T}_fetch gpurun_out/${T}_write gpurun_out/${T}_mfma gpurun_out/${T}_pmc_$i.json "$NAME" || exit 24
done
