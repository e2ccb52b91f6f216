# round 5: backward-kernel cost breakdown by compile-time variant (perf only; results wrong)
set -o pipefail
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; mkdir -p gpurun_out
T=${1:-r05j}
for v in base NO_B NO_C NO_DMA; do
  if [ $v = base ]; then L=dformer_amd/libdformer_hip.so; else L=dformer_amd/variants/lib_$v.so; fi
  DFM_LIB_PATH=$PWD/$L timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${T}_$v -o kt -- python3 tools/ffn_one.py 0 mlp 5 > gpurun_out/${T}_$v.log 2>&1 || exit 21
  echo "$v: $(grep ffn_bwd gpurun_out/${T}_$v/kt_kernel_stats.csv | cut -d, -f4)"
done
