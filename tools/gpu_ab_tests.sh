# GPU tests selected by $ABK, then a bench A/B over the env settings given as arguments
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests -x -q -m gpu -k "$ABK" --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/t.txt 2>&1; rc=$?; tail -2 gpurun_out/t.txt; [ $rc -eq 0 ] || exit 11
bash tools/gpu_abenv.sh "$@"
