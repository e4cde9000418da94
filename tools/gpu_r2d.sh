set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity_mmdopt.py tests/test_gpu_full_shape.py tests/test_gpu_configs0.py tests/test_gpu_free_run.py -v -s --timeout 240 --timeout-method thread -p no:cacheprovider > gpurun_out/r2d_tests.log 2>&1
rc=$?
grep -E "candidate|exact|runs part|PASSED|FAILED|passed|failed|Error" gpurun_out/r2d_tests.log | tail -40
for g in 1 2; do
  MPCMMD_GROUPS=$g timeout -k 10 120 python bench.py --cpu-seconds 0 --steps 40 > gpurun_out/r2d_bench_g$g.json 2> gpurun_out/r2d_bench_g$g.err || exit 1
  python -c "import json;d=json.load(open('gpurun_out/r2d_bench_g$g.json'));print($g, round(d['value'],2), {k:round(v,3) for k,v in d['kernels_ms_per_step'].items()})"
done
exit $rc
