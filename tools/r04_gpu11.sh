# mmd_opt parity + timing
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity_mmdopt.py tests/test_gpu_configs0.py tests/test_gpu_full_shape.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu > gpurun_out/t.log 2>&1; rc=$?; tail -3 gpurun_out/t.log; [ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" gpurun_out/t.log | head -20; exit 1; }
for wl in ${WORKLOADS:-mmd_opt}; do
  timeout -k 10 300 python bench.py --workload $wl --steps 40 --warmup 5 --cpu-seconds 0 --extra 0 > gpurun_out/ab_$wl.json || exit 1
  python -c "
import json
d=json.load(open('gpurun_out/ab_$wl.json')); print('$wl', round(d['value'],2), {k:round(v*1e3,1) for k,v in d['kernels_ms_per_step'].items()})"
done
