# LDS counters of the fused ConvFFN backward, per phase (DFM_FFN_SKIP masks isolate [A], [B], [C]):
# bash tools/ffn_lds_pmc.sh TAG STAGE   (on the GPU box)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=${1:-ffnlds}; S=${2:-0}
mkdir -p gpurun_out
for m in 0 6 5 3 7; do
  DFM_FFN_SKIP=$m timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_INSTS_LDS SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAIT_INST_LDS --kernel-include-regex convffn --output-format csv -d gpurun_out/${T}_m$m -o p -- python3 tools/ffn_bench.py $S 2 > /dev/null 2>&1 || exit 2
done
echo pmc-done
