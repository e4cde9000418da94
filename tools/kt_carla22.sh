# rocprofv3 kernel trace of the CARLA n = 22 bench (GPU box) and its two-stream
# overlap per outer iteration (tools/overlap.py, k_mother = one per iteration):
#   bash tools/kt_carla22.sh
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -s KILL 240 rocprofv3 --kernel-trace -d gpurun_out/kt22 -o run --output-format csv -- python3 bench.py --workload carla --carla-n 22 --steps 3 --warmup 1 > gpurun_out/kt22.log 2>&1 || exit 1
f=$(find gpurun_out/kt22 -name "*kernel_trace.csv" | head -1)
python3 tools/overlap.py $f 25 20 > gpurun_out/overlap_carla22.txt && cat gpurun_out/overlap_carla22.txt
gzip -c $f > gpurun_out/kt22_trace.csv.gz; find gpurun_out/kt22 -name "*kernel_trace.csv" -delete
