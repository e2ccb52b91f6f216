# PMC passes over tools/gemm_one.py for one GEMM shape (run on the GPU box):
#   bash tools/gemm_pmc.sh TAG M N K ak bk
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=$1; shift
mkdir -p gpurun_out
timeout -k 10 60 python3 tools/gemm_one.py "$@" 20 || exit 1
timeout -s KILL 90 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${T}_kt -o kt -- python3 tools/gemm_one.py "$@" 5 > /dev/null 2>&1 || exit 6
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS --output-format csv -d gpurun_out/${T}_p1 -o p1 -- python3 tools/gemm_one.py "$@" 3 > /dev/null 2>&1 || exit 2
timeout -s KILL 90 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_VMEM SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_VMEM --output-format csv -d gpurun_out/${T}_p2 -o p2 -- python3 tools/gemm_one.py "$@" 3 > /dev/null 2>&1 || exit 3
timeout -s KILL 90 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/${T}_p3 -o p3 -- python3 tools/gemm_one.py "$@" 3 > /dev/null 2>&1 || exit 4
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/${T}_p4 -o p4 -- python3 tools/gemm_one.py "$@" 3 > /dev/null 2>&1 || exit 5
echo pmc-done
