# Quick GPU iteration: mmd_opt parity tests + headline bench (per-kernel ms).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity_mmdopt.py -x -v --timeout 300 --timeout-method thread > gpurun_out/gpu_quick_tests.log 2>&1 && \
timeout -k 10 300 python bench.py --cpu-seconds 0 > gpurun_out/bench_quick.json 2> gpurun_out/bench_quick.err
