set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity_mmdopt.py tests/test_gpu_configs0.py tests/test_gpu_full_shape.py -v -s --timeout 240 --timeout-method thread -p no:cacheprovider > gpurun_out/r2g_tests.log 2>&1
rc=$?
grep -E "PASSED|FAILED|passed|failed|Error" gpurun_out/r2g_tests.log | tail -15
[ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python bench.py --cpu-seconds 0 --extra 0 > gpurun_out/r2g_bench.json 2> gpurun_out/r2g_bench.err
python -c "import json;d=json.load(open('gpurun_out/r2g_bench.json'));print(round(d['value'],2), {k:round(v,3) for k,v in d['kernels_ms_per_step'].items()})"
