set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -v -s --timeout 240 --timeout-method thread -p no:cacheprovider > gpurun_out/r2e_tests.log 2>&1
rc=$?
grep -E "runs part|exact|PASSED|FAILED|passed|failed|Error" gpurun_out/r2e_tests.log | tail -70
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/sweep_bench.py 64 4 32 > gpurun_out/r2e_sweep.log 2>&1; cat gpurun_out/r2e_sweep.log
timeout -k 10 120 python bench.py --cpu-seconds 0 --steps 40 > gpurun_out/r2e_bench.json 2> gpurun_out/r2e_bench.err
python -c "import json;d=json.load(open('gpurun_out/r2e_bench.json'));print(round(d['value'],2), {k:round(v,3) for k,v in d['kernels_ms_per_step'].items()})"
