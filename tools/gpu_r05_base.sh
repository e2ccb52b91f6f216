set -o pipefail
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 300 python -u bench.py --steps 40 --warmup 10 --no-cpu-baseline --table-out gpurun_out/r05a_step_table.json > gpurun_out/r05a_bench.log 2>&1 || exit 13
tail -1 gpurun_out/r05a_bench.log | cut -c1-400
timeout -k 10 300 python -u tools/ffn_kernels_bench.py 0 1 2 3 > gpurun_out/r05a_ffn.log 2>&1; echo ffn rc=$?
tail -60 gpurun_out/r05a_ffn.log
