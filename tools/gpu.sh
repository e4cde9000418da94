# One parametrised driver for the GPU box (run through gpurun):
#   bash tools/gpu.sh tests  [pytest selection...]   GPU tests (default: all -m gpu)
#   bash tools/gpu.sh smoke                          __graft_entry__.smoke()
#   bash tools/gpu.sh bench  TAG [bench args...]     bench.py -> gpurun_out/bench_TAG.json
#   bash tools/gpu.sh ab     CAND [bench args...]    bench.py with the default library, then MPCMMD_LIB=CAND
#   bash tools/gpu.sh prof   TAG [bench args...]     rocprofv3 stats + PMC passes (tools/prof.sh)
#   bash tools/gpu.sh round  TAG                     smoke && tests && bench && prof
# Several modes chain with "+": bash tools/gpu.sh "smoke+tests" ...  (arguments go to the last mode).
# Every GPU step has its own time limit; the chain stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
MODES=$1
shift

run_tests() {
  local sel=("$@")
  [ ${#sel[@]} -eq 0 ] && sel=(tests -m gpu)
  timeout -k 10 900 python -u -m pytest "${sel[@]}" -x -v -rA --timeout 300 --timeout-method thread \
    -p no:cacheprovider > gpurun_out/gpu_tests.log 2>&1
  local rc=$?
  grep -E "passed|failed|error" gpurun_out/gpu_tests.log | tail -2
  [ $rc -eq 0 ] || tail -40 gpurun_out/gpu_tests.log
  return $rc
}

run_bench() {
  local tag=$1
  shift
  timeout -k 10 400 python bench.py "$@" > gpurun_out/bench_$tag.json 2> gpurun_out/bench_$tag.err || {
    tail -20 gpurun_out/bench_$tag.err
    return 1
  }
  python -c "import json;d=json.load(open('gpurun_out/bench_$tag.json'));print('$tag', d['metric'][:20], round(d['value'],2), d.get('roofline',{}).get('frac'), {k:round(v,3) for k,v in d.get('kernels_ms_per_step',{}).items()})"
}

IFS='+' read -ra LIST <<< "$MODES"
for m in "${LIST[@]}"; do
  case $m in
    smoke) timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 && tail -1 gpurun_out/smoke.log || { tail -20 gpurun_out/smoke.log; exit 1; } ;;
    tests) run_tests "$@" || exit 1 ;;
    bench) run_bench "$@" || exit 1 ;;
    ab)
      cand=$1
      shift
      run_bench base "$@" || exit 1
      MPCMMD_LIB=$cand run_bench cand "$@" || exit 1 ;;
    prof) bash tools/prof.sh "$@" || exit 1 ;;
    round)
      tag=${1:-round}
      timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || exit 1
      run_tests || exit 1
      run_bench "default_$tag" || exit 1
      MPCMMD_GROUPS=1 bash tools/prof.sh "$tag" --extra 0 || exit 1 ;;
    *) echo "unknown mode $m"; exit 2 ;;
  esac
done
