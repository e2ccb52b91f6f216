# round 5 evidence: bench line + census table, rocprofv3 kernel stats, PMC of the dominant kernel and of
# the 7x7 depthwise / MFMA attention kernels
set -o pipefail
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; mkdir -p gpurun_out
T=${1:-r05e}
timeout -k 10 400 python -u bench.py --table-out gpurun_out/${T}_table.json > gpurun_out/${T}_bench.log 2>&1 || { tail -5 gpurun_out/${T}_bench.log; exit 11; }
tail -1 gpurun_out/${T}_bench.log | cut -c1-400
bash tools/gpu_prof.sh ${T} || exit 12
bash tools/gpu_pmc.sh ${T}dom gpurun_out/${T}_table.json || exit 13
bash tools/gpu_pmc_kernels.sh ${T}k gpurun_out/${T}_table.json "dw7_lds_wgrad_kernel" "dw_tile_fwd_kernel<unsigned short, 7, false" "dw_tile_fwd_kernel<unsigned short, 7, true" "attn_fwd_mfma_kernel" "attn_bwd_mfma_kernel" "dw3_stream_bwd_kernel" "dw3_stream_fwd_kernel" || exit 14
echo evidence done
