set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 && \
timeout -k 10 300 python bench.py --workload dynamic --cpu-seconds 0 --steps 20 --warmup 2 > gpurun_out/bench_dyn.json 2> gpurun_out/bench_dyn.err && \
timeout -k 10 300 python bench.py --workload cvar --cpu-seconds 0 > gpurun_out/bench_cvar.json 2> gpurun_out/bench_cvar.err
