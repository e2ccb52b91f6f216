# Usage (on the GPU box via gpurun): bash tools/ab_switches.sh TAG "VAR=val VAR2=val" ...
# One short bench.py run (30 timed steps, no census / CPU baseline) per environment setting.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=$1; shift
mkdir -p gpurun_out
i=0
for setting in "$@"; do
  i=$((i+1))
  env $setting timeout -k 10 300 python bench.py --steps 30 --warmup 10 --no-cpu-baseline --no-census > gpurun_out/${T}_ab$i.log 2>&1 || exit 20
  v=$(tail -1 gpurun_out/${T}_ab$i.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['step_ms_gpu']['median'])")
  echo "[$setting] $v" | tee -a gpurun_out/${T}_ab.txt
done
