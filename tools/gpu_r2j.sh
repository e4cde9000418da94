# QP change: beta-CEM tests (all n), then the mmd_opt bench.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity_mmdopt.py tests/test_gpu_full_shape.py tests/test_gpu_configs0.py tests/test_gpu_free_run.py -x -v --timeout 240 --timeout-method thread -p no:cacheprovider > gpurun_out/j_tests.log 2>&1 || { tail -30 gpurun_out/j_tests.log; exit 1; }
grep -E "passed|failed" gpurun_out/j_tests.log | tail -1
timeout -k 10 120 python bench.py --cpu-seconds 0 --extra 0 > gpurun_out/j_bench.json 2> gpurun_out/j_bench.err || exit 1
python -c "import json;d=json.load(open('gpurun_out/j_bench.json'));print(round(d['value'],2), {k:round(v,3) for k,v in d['kernels_ms_per_step'].items()})"
