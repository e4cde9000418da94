# Experiment arms on the mmd_opt bench, after a test selection.
#   bash tools/gpu_ab2.sh "ARM1 ARM2 ..." [test-selector|none] [bench args]
# An arm is an environment assignment (VAR=value), e.g. a switch or
# MPCMMD_LIB=mpc-mmd_amd/libmpcmmd_x.so; the default build runs first.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
ARMS=${1:-}
SEL=${2:-tests/test_gpu_parity_mmdopt.py}
BARGS=${3:-}
if [ "$SEL" != none ]; then
  timeout -k 10 500 python -u -m pytest $SEL -x -v --timeout 240 --timeout-method thread -p no:cacheprovider > gpurun_out/ab_tests.log 2>&1
  rc=$?
  grep -E "PASSED|FAILED|passed|failed|Error" gpurun_out/ab_tests.log | tail -15
  [ $rc -eq 0 ] || exit $rc
fi
i=0
for a in MPCMMD_DEFAULT=1 $ARMS; do
  env $a timeout -k 10 120 python bench.py --cpu-seconds 0 --extra 0 --steps 40 $BARGS > gpurun_out/ab_$i.json 2> gpurun_out/ab_$i.err || exit 1
  python -c "import json;d=json.load(open('gpurun_out/ab_$i.json'));print('$a', round(d['value'],2), {k:round(v,3) for k,v in d['kernels_ms_per_step'].items()})"
  i=$((i+1))
done
