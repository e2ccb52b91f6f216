# ring GEMM with the DMA issued as inline asm (variant build): parity, then default vs variant (NS 2 / 3)
set -o pipefail
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; mkdir -p gpurun_out
T=${1:-asmdma}; V=$GRAFT_REPO_ROOT/dformer_amd/variants/lib_asmdma.so
for ns in 2 3; do
  DFM_LIB_PATH=$V DFM_GLDS_NS=$ns timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
    tests/test_kernels_gpu.py -k "gemm or group or nmf" > gpurun_out/${T}_pytest_$ns.log 2>&1 || { tail -30 gpurun_out/${T}_pytest_$ns.log; exit 10; }
  tail -1 gpurun_out/${T}_pytest_$ns.log
done
DFM_LIB_PATH=$V DFM_GLDS_NS=3 timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_block_gpu.py > gpurun_out/${T}_pytest_blk.log 2>&1 || { tail -30 gpurun_out/${T}_pytest_blk.log; exit 10; }
tail -1 gpurun_out/${T}_pytest_blk.log
run() {  # tag, then env assignments
  tag=$1; shift
  env "$@" timeout -k 10 300 python -u bench.py --steps 60 --warmup 10 --no-cpu-baseline --no-census > gpurun_out/${T}_$tag.log 2>&1 || { tail -5 gpurun_out/${T}_$tag.log; exit 11; }
  echo "$tag: $(tail -1 gpurun_out/${T}_$tag.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["step_ms_gpu"])')"
}
for i in 1 2; do
  run base_$i DFM_GLDS_NS=2
  run asm2_$i DFM_LIB_PATH=$V DFM_GLDS_NS=2
  run asm3_$i DFM_LIB_PATH=$V DFM_GLDS_NS=3
done
