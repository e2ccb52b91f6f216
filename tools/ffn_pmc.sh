# PMC passes (one rocprofv3 run each, SQ counters only) over the fused ConvFFN kernels at one stage
set -o pipefail
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; mkdir -p gpurun_out
T=${1:-ffnpmc}; ST=${2:-0}; BR=${3:-mlp}
timeout -s KILL 60 rocprofv3 -L > gpurun_out/${T}_counters.txt 2>&1 || true
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS"
P2="SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES"
i=0
for P in "$P1" "$P2"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $P --output-format csv -d gpurun_out/${T}_p$i -o p -- python3 tools/ffn_one.py $ST $BR 3 > gpurun_out/${T}_p$i.log 2>&1 || { echo "pass $i failed"; tail -3 gpurun_out/${T}_p$i.log; exit 31; }
done
echo pmc done
