# round 5: fused ConvFFN parity (both modes) + per-stage timing + step A/B of the fused-forward mode
set -o pipefail
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; mkdir -p gpurun_out
T=${1:-r05r}
timeout -k 10 300 python -u -m pytest tests/test_convffn_gpu.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/${T}_convffn.log 2>&1 || { tail -20 gpurun_out/${T}_convffn.log; exit 11; }
tail -1 gpurun_out/${T}_convffn.log
timeout -k 10 300 python -u tools/ffn_kernels_bench.py 0 1 2 > gpurun_out/${T}_ffn.log 2>&1 || exit 12
grep -E "unfused" gpurun_out/${T}_ffn.log
bash tools/gpu_r05_ab.sh ${T}ab DFM_FUSED_FFN 0 fwd || exit 13
