# GPU-box check: microbench, GPU parity tests, a short bench.  Every GPU step
# has its own time limit and the chain stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
true && \
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 && \
timeout -k 10 300 python bench.py --cpu-seconds 0 > gpurun_out/bench.json 2> gpurun_out/bench.err
