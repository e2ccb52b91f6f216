# torch-side launch attribution + fresh kernel stats of the default bench
set -o pipefail
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; mkdir -p gpurun_out
T=${1:-prof2}
timeout -k 10 300 python -u tools/torchprof_copies.py > gpurun_out/${T}_copies.txt 2>&1 || { tail -20 gpurun_out/${T}_copies.txt; exit 10; }
head -30 gpurun_out/${T}_copies.txt
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_rp -o run -- python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-census > gpurun_out/${T}_bench.log 2>&1 || { tail -20 gpurun_out/${T}_bench.log; exit 11; }
tail -1 gpurun_out/${T}_bench.log
find gpurun_out/${T}_rp -name '*kernel_stats.csv' | head -1
