# mmd_opt iteration: parity tests (n = 5..32) + headline and configs[3] benches.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity_mmdopt.py tests/test_gpu_full_shape.py -x -v --timeout 300 --timeout-method thread > gpurun_out/gpu_quick_tests.log 2>&1 && \
timeout -k 10 300 python bench.py --cpu-seconds 0 > gpurun_out/bench_quick.json 2> gpurun_out/bench_quick.err && \
timeout -k 10 300 python bench.py --workload dynamic --cpu-seconds 0 --steps 20 --warmup 2 > gpurun_out/bench_dyn.json 2> gpurun_out/bench_dyn.err
