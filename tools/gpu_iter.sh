# Iteration pass: the named GPU test files (default: mmd_opt parity set), then the bench.
#   bash tools/gpu_iter.sh TAG "tests/a.py tests/b.py" "bench args"
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
TAG=${1:-it}
TESTS=${2:-"tests/test_gpu_parity_mmdopt.py tests/test_gpu_configs0.py tests/test_gpu_full_shape.py"}
BARGS=${3:-"--cpu-seconds 0 --extra 0"}
timeout -k 10 600 python -u -m pytest $TESTS -v -s --timeout 240 --timeout-method thread -p no:cacheprovider > gpurun_out/${TAG}_tests.log 2>&1
rc=$?
grep -E "PASSED|FAILED|passed|failed|Error|exact" gpurun_out/${TAG}_tests.log | tail -40
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py $BARGS > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || exit 1
python -c "
import json;d=json.load(open('gpurun_out/${TAG}_bench.json'))
print(round(d['value'],2), {k:round(v,3) for k,v in d['kernels_ms_per_step'].items()})
for k,v in d.get('extra_workloads',{}).items(): print(k, round(v['value'],2), {a:round(b,3) for a,b in v['kernels_ms_per_step'].items()})"
