# draws ahead in k_select: full GPU suite, then cvar / mmd_opt with MPCMMD_AHEAD=1 / 0
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu > gpurun_out/t.log 2>&1; rc=$?; tail -3 gpurun_out/t.log; [ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" gpurun_out/t.log | head -20; exit 1; }
for wl in cvar mmd_opt; do
  for a in 1 0; do
    MPCMMD_AHEAD=$a timeout -k 10 300 python bench.py --workload $wl --steps 60 --warmup 10 --cpu-seconds 0 --extra 0 > gpurun_out/ab_${wl}_$a.json || exit 1
    python -c "
import json
d=json.load(open('gpurun_out/ab_${wl}_$a.json')); print('$wl ahead=$a', round(d['value'],2), {k:round(v*1e3,1) for k,v in d['kernels_ms_per_step'].items()})"
  done
done
