# A/B of a variant build of the library (DFM_LIB_PATH) against the in-tree one on the default bench
#   bash tools/gpu_r05_lib_ab.sh TAG VARIANT_SO
set -o pipefail
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; mkdir -p gpurun_out
T=${1:-libab}; V=$2
for i in 1 2; do
  for lib in default $V; do
    if [ $lib = default ]; then unset DFM_LIB_PATH; else export DFM_LIB_PATH=$GRAFT_REPO_ROOT/$lib; fi
    timeout -k 10 300 python -u bench.py --steps 60 --warmup 10 --no-cpu-baseline --no-census > gpurun_out/${T}_$(basename $lib)_$i.log 2>&1 || { tail -5 gpurun_out/${T}_$(basename $lib)_$i.log; exit 11; }
    echo "$lib run $i: $(tail -1 gpurun_out/${T}_$(basename $lib)_$i.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["step_ms_gpu"])')"
  done
done
unset DFM_LIB_PATH
