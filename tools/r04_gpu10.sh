# per-iteration graphs: free-run parity with MPCMMD_GRAPH=1, cvar / mmd_opt A/B
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
MPCMMD_GRAPH=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_free_run.py tests/test_gpu_carla.py tests/test_gpu_handle_lifecycle.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu > gpurun_out/t.log 2>&1; rc=$?; tail -3 gpurun_out/t.log; [ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" gpurun_out/t.log | head -20; exit 1; }
for g in 0 1; do
  for wl in cvar; do
    MPCMMD_GRAPH=$g timeout -k 10 300 python bench.py --workload $wl --steps 100 --warmup 5 --cpu-seconds 0 --extra 0 > gpurun_out/ab_${wl}_g$g.json || exit 1
    python -c "
import json
d=json.load(open('gpurun_out/ab_${wl}_g$g.json')); print('$wl graph=$g', round(d['value'],2), round(d['ms_per_step']*1e3,1))"
  done
done
