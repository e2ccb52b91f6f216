# round 5: fused ConvFFN parity + per-stage timing + whole-step A/B (op-level chain vs fused)
set -o pipefail
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; mkdir -p gpurun_out
T=${1:-r05l}
timeout -k 10 300 python -u -m pytest tests/test_convffn_gpu.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/${T}_convffn.log 2>&1 || { tail -20 gpurun_out/${T}_convffn.log; exit 11; }
tail -1 gpurun_out/${T}_convffn.log
timeout -k 10 300 python -u tools/ffn_kernels_bench.py 0 1 2 > gpurun_out/${T}_ffn.log 2>&1 || exit 12
grep -E "unfused" gpurun_out/${T}_ffn.log
for f in 0 1; do
  DFM_FUSED_FFN=$f timeout -k 10 300 python -u bench.py --steps 30 --warmup 10 --no-cpu-baseline --table-out gpurun_out/${T}_table_f$f.json > gpurun_out/${T}_bench_f$f.log 2>&1 || exit 13
  echo "fused=$f: $(tail -1 gpurun_out/${T}_bench_f$f.log | cut -c1-200)"
done
