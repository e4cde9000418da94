# GPU box: selected GPU tests, then an A/B of library variants on the headline bench.
#   bash tools/gpu_tab.sh TAG "tests/test_a.py tests/test_b.py" "base=MPCMMD_LIB=mpc-mmd_amd/libmpcmmd_base.so" "new=X=1"
# Tests "-" = none.  Every GPU step has its own time limit; the chain stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
TAG=$1; TESTS=$2; shift 2
if [ "$TESTS" != "-" ]; then
  timeout -k 10 600 python -u -m pytest $TESTS -v -s --timeout 240 --timeout-method thread -p no:cacheprovider > gpurun_out/${TAG}_tests.log 2>&1
  rc=$?
  grep -E "PASSED|FAILED|passed|failed|Error" gpurun_out/${TAG}_tests.log | tail -25
  [ $rc -eq 0 ] || exit $rc
fi
[ $# -eq 0 ] && exit 0
bash tools/gpu_ab.sh "$@"
