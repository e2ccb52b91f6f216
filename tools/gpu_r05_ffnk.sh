# isolated ConvFFN kernel timings, in-tree build vs a variant build
set -o pipefail
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; mkdir -p gpurun_out
T=${1:-ffnk}
timeout -k 10 300 python -u tools/ffn_kernels_bench.py 0 1 2 3 > gpurun_out/${T}_new.txt 2>&1 || { tail -20 gpurun_out/${T}_new.txt; exit 10; }
if [ -n "$2" ]; then
  DFM_LIB_PATH=$GRAFT_REPO_ROOT/$2 timeout -k 10 300 python -u tools/ffn_kernels_bench.py 0 1 2 3 > gpurun_out/${T}_old.txt 2>&1 || { tail -20 gpurun_out/${T}_old.txt; exit 11; }
fi
grep -E "dw3" gpurun_out/${T}_*.txt
