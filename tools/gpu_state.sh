# Session-start state check: every GPU test, the default bench with all workloads (no CPU leg), rocprof kernel stats.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -v -s --timeout 240 --timeout-method thread -p no:cacheprovider > gpurun_out/st_tests.log 2>&1
rc=$?
grep -E "PASSED|FAILED|passed|failed|Error" gpurun_out/st_tests.log | tail -60
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --cpu-seconds 0 > gpurun_out/st_bench.json 2> gpurun_out/st_bench.err && \
python -c "import json;d=json.load(open('gpurun_out/st_bench.json'));print(round(d['value'],2), {k:round(v,3) for k,v in d['kernels_ms_per_step'].items()}); [print(k, round(v['value'],2), {a:round(b,3) for a,b in v['kernels_ms_per_step'].items()}) for k,v in d['extra_workloads'].items()]" && \
timeout -s KILL 240 rocprofv3 --kernel-trace --stats -d gpurun_out/st_prof -o run --output-format csv -- python3 bench.py --steps 20 --warmup 2 --profile-steps 20 --cpu-seconds 0 --extra 0 > gpurun_out/st_prof.log 2>&1
