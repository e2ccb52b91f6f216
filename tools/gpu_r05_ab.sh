# A/B of one environment switch on the default bench (alternating runs):
#   bash tools/gpu_r05_ab.sh TAG VAR [VALUE_A VALUE_B]   (default values 0 1)
set -o pipefail
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; mkdir -p gpurun_out
T=${1:-ab}; V=${2:?switch name}; A=${3:-0}; B=${4:-1}
for i in 1 2; do
  for v in $A $B; do
    env $V=$v timeout -k 10 300 python -u bench.py --steps 60 --warmup 10 --no-cpu-baseline --no-census > gpurun_out/${T}_${v}_$i.log 2>&1 || { tail -5 gpurun_out/${T}_${v}_$i.log; exit 11; }
    echo "$V=$v run $i: $(tail -1 gpurun_out/${T}_${v}_$i.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["step_ms_gpu"])')"
  done
done
