# Round checkpoint on the GPU box: smoke, every GPU test, the default bench
# (all workloads + CPU baseline), then the rocprofv3 passes of tools/prof.sh.
#   bash tools/gpu_round.sh TAG
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TAG=${1:-round}
mkdir -p gpurun_out
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 && \
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/gpu_tests.log 2>&1 && \
grep -E "passed|failed" gpurun_out/gpu_tests.log | tail -2 && \
timeout -k 10 400 python bench.py > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err && \
MPCMMD_GROUPS=1 bash tools/prof.sh $TAG --extra 0
