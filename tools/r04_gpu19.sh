# two-wave sampler experiment (MPCMMD_BSAMPLE3=1): full-shape parity, then mmd_opt A/B
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
MPCMMD_BSAMPLE3=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_full_shape.py tests/test_gpu_handle_lifecycle.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu -k "mmd_opt or lifecycle or constants or front" > gpurun_out/t3.log 2>&1; rc=$?; tail -3 gpurun_out/t3.log; [ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" gpurun_out/t3.log | head -20; exit 1; }
for e in 1 0; do
  MPCMMD_BSAMPLE3=$e timeout -k 10 300 python bench.py --workload mmd_opt --steps 60 --warmup 5 --cpu-seconds 0 --extra 0 > gpurun_out/ab3_$e.json || exit 1
  python -c "
import json
d=json.load(open('gpurun_out/ab3_$e.json')); print('bsample3=$e', round(d['value'],2), {k:round(v*1e3,1) for k,v in d['kernels_ms_per_step'].items() if k in ('bsample','bselect','bkernel','bqp','belite','bgen')})"
done
MPCMMD_BSAMPLE3=1 MPCMMD_GROUPS=1 timeout -k 10 300 python bench.py --workload mmd_opt --steps 40 --warmup 5 --cpu-seconds 0 --extra 0 > gpurun_out/ab3_g1.json && python -c "
import json
d=json.load(open('gpurun_out/ab3_g1.json')); print('bsample3=1 groups=1', round(d['value'],2), round(d['kernels_ms_per_step']['bsample']*1e3,1))"
