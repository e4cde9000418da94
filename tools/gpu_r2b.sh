# round 2: full GPU test suite, then the headline bench (groups 1 and 2)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -v -s --timeout 240 --timeout-method thread -p no:cacheprovider > gpurun_out/r2b_tests.log 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR|passed|failed" gpurun_out/r2b_tests.log | tail -60
[ $rc -eq 0 ] || exit $rc
for g in 1 2; do
  MPCMMD_GROUPS=$g timeout -k 10 120 python bench.py --cpu-seconds 0 --steps 40 > gpurun_out/r2b_bench_g$g.json 2> gpurun_out/r2b_bench_g$g.err || exit 1
  python -c "import json;d=json.load(open('gpurun_out/r2b_bench_g$g.json'));print($g, round(d['value'],2), {k:round(v,3) for k,v in d['kernels_ms_per_step'].items()})"
done
