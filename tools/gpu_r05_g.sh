# round 5: tall short-K GEMMs (K <= 128) against hipBLASLt on the DFormer-B step's shapes
set -o pipefail
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; mkdir -p gpurun_out
T=${1:-r05g}
timeout -k 10 500 python -u tools/gemm_sweep.py --no-splits --out gpurun_out/${T}_sweep.json > gpurun_out/${T}_sweep.log 2>&1 || { tail -5 gpurun_out/${T}_sweep.log; exit 11; }
timeout -k 10 400 python -u tools/gemm_blas.py --sweep gpurun_out/${T}_sweep.json --max-k 128 --out gpurun_out/${T}_blas.json > gpurun_out/${T}_blas.txt 2>&1 || { tail -5 gpurun_out/${T}_blas.txt; exit 12; }
cat gpurun_out/${T}_blas.txt
