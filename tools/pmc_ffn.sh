# PMC passes over tools/ffn_kernels_bench.py (stage S) for kernels matching REGEX (run on the GPU box):
#   bash tools/pmc_ffn.sh TAG S 'dw3_stream_bwd|dw_tile_fwd'
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; mkdir -p gpurun_out
T=$1; S=$2; RX=$3
timeout -s KILL 120 rocprofv3 --kernel-trace --stats --kernel-include-regex "$RX" --output-format csv -d gpurun_out/${T}_kt -o kt -- python3 tools/ffn_kernels_bench.py $S > /dev/null 2>&1 || exit 6
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_ACTIVE_INST_VALU --kernel-include-regex "$RX" --output-format csv -d gpurun_out/${T}_p1 -o p1 -- python3 tools/ffn_kernels_bench.py $S > /dev/null 2>&1 || exit 2
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VMEM SQ_INSTS_LDS SQ_INSTS_SALU SQ_INST_CYCLES_VMEM SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE --kernel-include-regex "$RX" --output-format csv -d gpurun_out/${T}_p2 -o p2 -- python3 tools/ffn_kernels_bench.py $S > /dev/null 2>&1 || exit 3
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "$RX" --output-format csv -d gpurun_out/${T}_p3 -o p3 -- python3 tools/ffn_kernels_bench.py $S > /dev/null 2>&1 || exit 4
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "$RX" --output-format csv -d gpurun_out/${T}_p4 -o p4 -- python3 tools/ffn_kernels_bench.py $S > /dev/null 2>&1 || exit 5
echo pmc-done
