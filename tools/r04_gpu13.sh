# per-iteration graphs at small batches: configs0 A/B
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
for g in 0 1; do
  MPCMMD_GRAPH=$g timeout -k 10 300 python bench.py --workload configs0 --steps 40 --warmup 25 --cpu-seconds 0 --extra 0 > gpurun_out/ab_c0_g$g.json || exit 1
  python -c "
import json
d=json.load(open('gpurun_out/ab_c0_g$g.json')); print('configs0 graph=$g', round(d['value'],2), round(d['ms_per_step'],3))"
done
