# Usage (on the GPU box via gpurun): bash tools/gpu_round3.sh TAG
# Round-3 evidence: GPU parity suite + smoke; a census bench (step table -> dominant kernel); unfiltered
# PMC passes (FETCH_SIZE, WRITE_SIZE, MFMA busy) -> per-kernel traffic / MFMA-busy for the dominant
# kernel and the north star's kernels; the final bench line (reads profiles/r03_pmc_dominant.json);
# rocprofv3 kernel trace + stats of the default step.
set -o pipefail
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; mkdir -p gpurun_out
T=${1:-r03z}
bash tools/gpu_tests.sh ${T} || exit 11
timeout -k 10 300 python -u bench.py --steps 20 --warmup 10 --no-cpu-baseline --table-out gpurun_out/${T}_step_table.json > gpurun_out/${T}_census.log 2>&1 || exit 12
B="bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-census --eager"
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/${T}_fetch -o f -- python3 $B > gpurun_out/${T}_fetch.log 2>&1 || exit 21
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/${T}_write -o w -- python3 $B > gpurun_out/${T}_write.log 2>&1 || exit 22
timeout -s KILL 300 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/${T}_mfma -o m -- python3 $B > gpurun_out/${T}_mfma.log 2>&1 || exit 23
python3 tools/pmc_kernels.py gpurun_out/${T}_step_table.json gpurun_out/${T}_fetch gpurun_out/${T}_write gpurun_out/${T}_mfma gpurun_out/${T}_pmc \
  "attn_fwd=attn_fwd_mfma" "attn_bwd=attn_bwd_mfma" "fwd_gemm=gemm_glds_kernel<64, 128, 4, 2, true, true" \
  "fc1_smallk=gemm_kernel<unsigned short, 128, 128, 8, 2, 32, true, true" "wgrad_group=gemm_group_kernel" \
  "dw3_bwd=dw3_stream_bwd" "dgrad_smallk=gemm_kernel<unsigned short, 128, 128, 8, 2, 32, true, false" > gpurun_out/${T}_pmc.log 2>&1 || exit 24
cp gpurun_out/${T}_pmc_dominant.json profiles/r03_pmc_dominant.json
timeout -k 10 400 python -u bench.py --table-out gpurun_out/${T}_step_table_final.json > gpurun_out/${T}_bench.log 2>&1 || exit 13
tail -1 gpurun_out/${T}_bench.log | cut -c1-300
bash tools/gpu_prof.sh ${T} || exit 14
echo done
