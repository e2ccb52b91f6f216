# PMC passes over tools/ffn_bench.py (run on the GPU box): bash tools/ffn_pmc.sh TAG STAGE
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=${1:-ffn}; S=${2:-0}
mkdir -p gpurun_out
timeout -k 10 120 python3 tools/ffn_bench.py $S 20 || exit 1
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS --output-format csv -d gpurun_out/${T}_p1 -o p1 -- python3 tools/ffn_bench.py $S 3 > /dev/null 2>&1 || exit 2
timeout -s KILL 90 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_MFMA SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_INSTS_VMEM SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_VMEM --output-format csv -d gpurun_out/${T}_p2 -o p2 -- python3 tools/ffn_bench.py $S 3 > /dev/null 2>&1 || exit 3
echo pmc-done
