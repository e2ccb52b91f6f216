# round 5: attention / depthwise parity after the XCD-aware block orders, bench line + census table,
# PMC traffic of the 7x7 depthwise and MFMA attention kernels
set -o pipefail
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; mkdir -p gpurun_out
T=${1:-r05s}
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py -x -q -k "attn or dw or pool" --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/${T}_t.log 2>&1 || { tail -30 gpurun_out/${T}_t.log; exit 11; }
tail -1 gpurun_out/${T}_t.log
timeout -k 10 600 python -u -m pytest tests/test_block_gpu.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/${T}_tb.log 2>&1 || { tail -30 gpurun_out/${T}_tb.log; exit 12; }
tail -1 gpurun_out/${T}_tb.log
timeout -k 10 400 python -u bench.py --no-cpu-baseline --table-out gpurun_out/${T}_table.json > gpurun_out/${T}_bench.log 2>&1 || { tail -5 gpurun_out/${T}_bench.log; exit 13; }
tail -1 gpurun_out/${T}_bench.log | cut -c1-300
bash tools/gpu_pmc_kernels.sh ${T}k gpurun_out/${T}_table.json "dw7_lds_wgrad_kernel" "attn_fwd_mfma_kernel" "attn_bwd_mfma_kernel" || exit 14
for i in 1 2 3; do python3 -c "import json; d=json.load(open('gpurun_out/${T}k_$i.json')); print(d['kernel'][:60], d['traffic_over_algorithmic'], d['algorithmic_frac_of_8TBs'], d['census_ms_per_launch'])"; done
