# BASELINE configs 2 and 5 on one GPU (bench.py lines), after the default step
set -o pipefail
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; mkdir -p gpurun_out
T=${1:-cfg}
timeout -k 10 300 python -u bench.py --arch DFormer-Tiny --batch 8 --no-cpu-baseline --table-out gpurun_out/${T}_config2_table.json > gpurun_out/${T}_config2.log 2>&1 || exit 21
echo "config2:"; tail -1 gpurun_out/${T}_config2.log | cut -c1-260
timeout -k 10 400 python -u bench.py --arch DFormer-Large --decoder MLPDecoder --height 530 --width 730 --ncls 37 --dtype fp16 --steps 30 --warmup 10 --no-cpu-baseline --table-out gpurun_out/${T}_config5_table.json > gpurun_out/${T}_config5.log 2>&1 || exit 22
echo "config5:"; tail -1 gpurun_out/${T}_config5.log | cut -c1-260
