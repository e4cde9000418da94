set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity_baseline.py -x -q --timeout 200 --timeout-method thread > gpurun_out/cv_tests.log 2>&1 && \
timeout -k 10 300 python bench.py --workload cvar --cpu-seconds 0 --steps 100 > gpurun_out/bench_cvar.json 2> gpurun_out/bench_cvar.err
