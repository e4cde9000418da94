set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_carla.py -x -v -rA --timeout 400 --timeout-method thread -p no:cacheprovider > gpurun_out/gpu_carla.log 2>&1
rc=$?
grep -E "passed|failed|error" gpurun_out/gpu_carla.log | tail -3
[ $rc -eq 0 ] || { tail -60 gpurun_out/gpu_carla.log; exit 1; }
timeout -k 10 300 python bench.py --workload carla --steps 10 --warmup 2 > gpurun_out/bench_carla.json 2> gpurun_out/bench_carla.err || { tail -30 gpurun_out/bench_carla.err; exit 1; }
cat gpurun_out/bench_carla.json
bash tools/gpu.sh tests
