# depthwise / reduction changes: their GPU tests, the ConvFFN shapes' 3x3 timings, one bench line
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests -x -q -m gpu -k "${DWK:-dw or dwconv or block or ffn or deferred or partial}" --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/dw_tests.txt 2>&1; rc=$?; tail -3 gpurun_out/dw_tests.txt; [ $rc -eq 0 ] || exit 11
timeout -k 10 200 python -u tools/dw3_geom_sweep.py > gpurun_out/dw3_built.txt 2>&1 || exit 12
cat gpurun_out/dw3_built.txt
timeout -k 10 300 python -u bench.py > gpurun_out/bench_dw.log 2>&1 || exit 13
tail -1 gpurun_out/bench_dw.log | cut -c1-300
