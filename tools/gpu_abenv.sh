# bench A/B over env settings given as arguments (each "VAR=val VAR2=val" or "X=1" for the default),
# alternated twice on one box
set -o pipefail
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; mkdir -p gpurun_out
for i in 1 2; do
for cfg in "$@"; do
env $cfg timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-census > gpurun_out/abenv.log 2>&1 || exit 13
echo "$cfg $(tail -1 gpurun_out/abenv.log | grep -o '"value": [0-9.]*, ')$(tail -1 gpurun_out/abenv.log | grep -o '"ms_per_step": [0-9.]*')"
done; done
