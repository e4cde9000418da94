# round 2: mmd_opt parity tests + bench with 1/2/3 candidate groups
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity_mmdopt.py tests/test_gpu_full_shape.py -x -v --timeout 200 --timeout-method thread > gpurun_out/r2a_tests.log 2>&1
rc=$?
tail -3 gpurun_out/r2a_tests.log
[ $rc -eq 0 ] || exit $rc
for g in 1 2 3; do
  MPCMMD_GROUPS=$g timeout -k 10 120 python bench.py --cpu-seconds 0 --steps 40 > gpurun_out/r2a_bench_g$g.json 2> gpurun_out/r2a_bench_g$g.err || exit 1
  python -c "import json;d=json.load(open('gpurun_out/r2a_bench_g$g.json'));print($g, round(d['value'],2), {k:round(v,3) for k,v in d['kernels_ms_per_step'].items()})"
done
