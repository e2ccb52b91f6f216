# A/B/n of environment switches on the default bench (alternating rounds):
#   bash tools/gpu_r05_abn.sh TAG "VAR=a VAR=b ..." ["VAR2=a VAR2=b ..."]
set -o pipefail
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; mkdir -p gpurun_out
T=$1; shift
for set in "$@"; do
  for i in 1 2; do
    for kv in $set; do
      tag=${T}_$(echo $kv | tr '=' '_')_$i
      env $kv timeout -k 10 300 python -u bench.py --steps 60 --warmup 10 --no-cpu-baseline --no-census > gpurun_out/$tag.log 2>&1 || { tail -5 gpurun_out/$tag.log; exit 11; }
      echo "$kv run $i: $(tail -1 gpurun_out/$tag.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["step_ms_gpu"])')"
    done
  done
done
