set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_carla.py -x -v -rA --timeout 400 --timeout-method thread -p no:cacheprovider > gpurun_out/gpu_carla.log 2>&1
rc=$?
grep -E "passed|failed|error" gpurun_out/gpu_carla.log | tail -3
[ $rc -eq 0 ] || { tail -60 gpurun_out/gpu_carla.log; exit 1; }
bash tools/gpu.sh tests
