# Per-launch durations (rocprofv3 kernel trace, one candidate group) of the
# beta-CEM kernels for the default library and any MPCMMD_LIB variants given:
#   bash tools/kt_variants.sh [mpc-mmd_amd/libmpcmmd_X.so ...]
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
for lib in mpc-mmd_amd/libmpcmmd.so "$@"; do
  tag=$(basename $lib .so)
  MPCMMD_LIB=$lib MPCMMD_GROUPS=1 timeout -s KILL 120 rocprofv3 --kernel-trace -d gpurun_out/kt_$tag -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --profile-steps 1 --extra 0 --cpu-seconds 0 > gpurun_out/kt_$tag.log 2>&1 || exit 1
  echo "== $tag"; python tools/ktrace.py gpurun_out/kt_$tag/run_kernel_trace.csv ${KT_FILTER:-bkernel bdirect}
done
