# BASELINE configs 2 and 5 on one GPU with the census on (roofline filled), final round-5 tree
set -o pipefail
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 400 python -u bench.py --arch DFormer-Tiny --batch 8 --no-cpu-baseline > gpurun_out/r05_config2.log 2>&1 || { tail -5 gpurun_out/r05_config2.log; exit 11; }
tail -1 gpurun_out/r05_config2.log | cut -c1-240
timeout -k 10 500 python -u bench.py --arch DFormer-Large --decoder MLPDecoder --ncls 37 --height 530 --width 730 --dtype fp16 --steps 30 --warmup 10 --no-cpu-baseline > gpurun_out/r05_config5.log 2>&1 || { tail -5 gpurun_out/r05_config5.log; exit 12; }
tail -1 gpurun_out/r05_config5.log | cut -c1-240
