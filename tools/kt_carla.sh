# rocprofv3 kernel trace of the CARLA bench under each setting (GPU box):
#   bash tools/kt_carla.sh N TAG "ENV=a ..." [TAG2 "ENV=b ..."]...
# Writes gpurun_out/kt_<TAG>/run_kernel_stats.csv and prints the per-tick kernel sums.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
N=$1
shift
while [ $# -ge 2 ]; do
  tag=$1; setting=$2; shift 2
  mkdir -p gpurun_out/kt_$tag
  env $setting timeout -s KILL 300 rocprofv3 --kernel-trace --stats -d gpurun_out/kt_$tag -o run --output-format csv -- \
    python3 bench.py --workload carla --carla-n $N --steps 4 --warmup 1 > gpurun_out/kt_$tag.log 2>&1 || { tail -5 gpurun_out/kt_$tag.log; exit 1; }
  f=$(find gpurun_out/kt_$tag -name "*kernel_stats.csv" | head -1)
  python3 - "$f" "$tag" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
tot = sum(float(r["TotalDurationNs"]) for r in rows) / 1e6
print(sys.argv[2], "total kernel ms %.1f" % tot)
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:12]:
    print("   %-50s calls %5d avg %7.1f us total %7.2f ms" % (r["Name"][:50].replace("mpcmmd::(anonymous namespace)::", ""), int(r["Calls"]), float(r["AverageNs"]) / 1e3, float(r["TotalDurationNs"]) / 1e6))
PY
done
