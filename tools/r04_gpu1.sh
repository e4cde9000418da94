set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 60 ./tools/microbench > gpurun_out/microbench.txt 2>&1 && cat gpurun_out/microbench.txt && \
bash tools/gpu.sh smoke+tests && \
bash tools/gpu.sh bench r04a
