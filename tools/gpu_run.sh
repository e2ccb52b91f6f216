# One parametrised GPU-box script (run through gpurun; every GPU step under its own timeout, steps
# chained so the first failure ends the call). Usage:
#   bash tools/gpu_run.sh suite  TAG [PYTEST_K]   full -m gpu suite (or the tests matching -k) + smoke()
#   bash tools/gpu_run.sh bench  TAG [ARGS...]    one default bench line (+ step table) with extra bench.py args
#   bash tools/gpu_run.sh libab  TAG LIB.so       bench A/B: in-tree library vs a variant build, alternated twice
#   bash tools/gpu_run.sh envab  TAG "A=1" "B=2"  bench A/B over environment settings, alternated twice
#   bash tools/gpu_run.sh py     TAG SCRIPT [ARGS...]  one diagnostic python script (output under gpurun_out/)
#   bash tools/gpu_run.sh final  TAG              round record: suite, smoke, bench + table, PMC passes over the
#                                                 census-dominant kernels, rocprofv3 --stats, kernel trace, configs 2 / 5
#   bash tools/gpu_run.sh record TAG              the same without the suite
# Every library load prints its path and build tag (dformer_amd._lib), so a variant run names what it loaded.
set -o pipefail
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; mkdir -p gpurun_out
CMD=$1; T=${2:-run}; shift 2

line() {  # value / ms of the last bench line in $1
  tail -1 "$1" | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d.get("lib_tag"), (d.get("roofline") or {}).get("frac"))'
}

suite() {
  local k=()
  [ -n "$1" ] && k=(-k "$1")
  timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider "${k[@]}" > gpurun_out/${T}_pytest.log 2>&1 || { tail -40 gpurun_out/${T}_pytest.log; return 10; }
  tail -2 gpurun_out/${T}_pytest.log
  timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${T}_smoke.log 2>&1 || { tail -20 gpurun_out/${T}_smoke.log; return 11; }
  tail -1 gpurun_out/${T}_smoke.log
}

case $CMD in
  suite) suite "$1" ;;
  bench)
    timeout -k 10 400 python -u bench.py --table-out gpurun_out/${T}_step_table.json "$@" > gpurun_out/${T}_bench.log 2>&1 || { tail -20 gpurun_out/${T}_bench.log; exit 12; }
    tail -1 gpurun_out/${T}_bench.log | cut -c1-1500 ;;
  libab)
    V=$1
    for i in 1 2; do
      for lib in default $V; do
        if [ $lib = default ]; then unset DFM_LIB_PATH; else export DFM_LIB_PATH=$GRAFT_REPO_ROOT/$lib; fi
        L=gpurun_out/${T}_$(basename $lib)_$i.log
        timeout -k 10 300 python -u bench.py --steps 60 --warmup 10 --no-cpu-baseline --no-census > $L 2>&1 || { tail -5 $L; exit 13; }
        echo "$lib run $i: $(line $L)"
      done
    done ;;
  envab)
    for i in 1 2; do
      for cfg in "$@"; do
        L=gpurun_out/${T}_$i.log
        env $cfg timeout -k 10 300 python -u bench.py --steps 60 --warmup 10 --no-cpu-baseline --no-census > $L 2>&1 || { tail -5 $L; exit 14; }
        echo "$cfg run $i: $(line $L)"
      done
    done ;;
  py)
    S=$1; shift
    timeout -k 10 600 python -u "$S" "$@" > gpurun_out/${T}_py.log 2>&1; rc=$?
    tail -40 gpurun_out/${T}_py.log; exit $rc ;;
  final|record)  # record = final without the suite (run it as its own call when a box's limit is tight)
    [ $CMD = final ] && { suite || exit $?; }
    timeout -k 10 400 python -u bench.py --table-out gpurun_out/${T}_step_table.json > gpurun_out/${T}_bench.log 2>&1 || exit 12
    tail -1 gpurun_out/${T}_bench.log | cut -c1-600
    bash tools/gpu_pmc.sh ${T} gpurun_out/${T}_step_table.json || exit 15
    timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${T}_stats -o ${T} -- python3 bench.py --no-cpu-baseline > gpurun_out/${T}_stats.log 2>&1 || exit 16
    rm -f gpurun_out/${T}_stats/${T}_kernel_trace.csv
    bash tools/gpu_prof.sh ${T} || exit 17
    rm -f gpurun_out/${T}_prof/${T}_kernel_trace.csv
    bash tools/gpu_configs.sh ${T} || exit 18 ;;
  *) echo "unknown command $CMD"; exit 2 ;;
esac
