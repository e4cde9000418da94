# Per-launch durations of the cvar workload's kernels (rocprofv3 kernel trace)
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
timeout -s KILL 120 rocprofv3 --kernel-trace -d gpurun_out/ktc -o run --output-format csv -- python3 bench.py --workload cvar --steps 4 --warmup 1 --profile-steps 1 --extra 0 --cpu-seconds 0 > gpurun_out/ktc.log 2>&1 && python tools/ktrace.py gpurun_out/ktc/run_kernel_trace.csv beta risk gamma front select
