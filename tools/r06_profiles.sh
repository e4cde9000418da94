# Round-6 profile collection (GPU box): bench line, rocprofv3 stats + PMC passes for
# mmd_opt and cvar, the CARLA kernel trace; bulky per-dispatch CSVs dropped so
# gpurun_out stays under the copy-back limit.   bash tools/r06_profiles.sh TAG
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
TAG=$1
( set -o pipefail
  bash tools/gpu.sh bench default_$TAG && \
  MPCMMD_GROUPS=1 bash tools/prof.sh $TAG --extra 0 && \
  MPCMMD_GROUPS=1 bash tools/prof.sh ${TAG}_cvar --workload cvar && \
  mkdir -p gpurun_out/kt_carla_$TAG && \
  timeout -s KILL 300 rocprofv3 --kernel-trace --stats -d gpurun_out/kt_carla_$TAG -o run --output-format csv -- \
    python3 bench.py --workload carla --steps 10 --warmup 2 > gpurun_out/kt_carla_$TAG.log 2>&1 )
rc=$?
# summaries on the box, then the raw per-dispatch CSVs dropped (copy-back limit 64 MiB)
[ $rc -eq 0 ] && PROFILES_OUT=gpurun_out/profiles_$TAG python3 tools/collect_profiles.py $TAG
rm -rf gpurun_out/prof_$TAG gpurun_out/prof_${TAG}_cvar
find gpurun_out -name "*kernel_trace.csv" -delete
find gpurun_out -name "*counter_collection.csv" -delete
du -sh gpurun_out
exit $rc
