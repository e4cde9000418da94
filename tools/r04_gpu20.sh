# mmd_opt candidate-group offset experiment (MPCMMD_GROUP_LAG)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
for lag in 0 -1 1 2 3 4 7; do
  MPCMMD_GROUP_LAG=$lag timeout -k 10 300 python bench.py --workload mmd_opt --steps 60 --warmup 5 --cpu-seconds 0 --extra 0 > gpurun_out/lag_$lag.json || exit 1
  python -c "
import json
d=json.load(open('gpurun_out/lag_$lag.json')); print('lag $lag', round(d['value'],2), round(d['ms_per_step'],3))"
done
