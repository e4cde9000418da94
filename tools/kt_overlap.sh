cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -s KILL 200 rocprofv3 --kernel-trace -d gpurun_out/kt2 -o run --output-format csv -- python3 bench.py --steps 6 --warmup 2 --profile-steps 1 --extra 0 --cpu-seconds 0 > gpurun_out/kt2.log 2>&1 || exit 1
f=$(find gpurun_out/kt2 -name "*kernel_trace.csv" | head -1)
python3 tools/overlap.py $f 2 6 > gpurun_out/overlap_mmdopt.txt && cat gpurun_out/overlap_mmdopt.txt
gzip -c $f > gpurun_out/kt2_trace.csv.gz; find gpurun_out/kt2 -name "*kernel_trace.csv" -delete
