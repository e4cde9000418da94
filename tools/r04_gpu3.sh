set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 300 python tools/carla_timing.py 10 8 2>&1 | tee gpurun_out/carla_timing.txt && \
timeout -k 10 300 python tools/carla_timing.py 22 6 2>&1 | tee -a gpurun_out/carla_timing.txt && \
timeout -k 10 600 python -u -m pytest tests/test_gpu_carla.py -x -q --timeout 400 --timeout-method thread -p no:cacheprovider > gpurun_out/gpu_carla_graph.log 2>&1; tail -3 gpurun_out/gpu_carla_graph.log
