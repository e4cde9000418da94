# Same-process-per-setting A/B of one CARLA mmd solve's wall time (tools/carla_enqueue.py; GPU box):
#   bash tools/carla_ab2.sh N "ENV=a ..." "ENV=b ..." ...   (each setting twice, interleaved)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
N=$1
shift
for rep in 1 2; do
  for setting in "$@"; do
    r=$(env $setting timeout -k 10 120 python tools/carla_enqueue.py $N 4 | tail -2 | awk '{s += $NF + 0} END {printf "%.2f", s / 2}') || exit 1
    echo "$setting => solve ${r} ms"
  done
done
