# MFMA-shadow probe + k_bsample interleave: parity, mmd_opt A/B against a base library
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 60 ./tools/mfma_overlap > gpurun_out/overlap.log 2>&1; rc=$?; cat gpurun_out/overlap.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity_mmdopt.py tests/test_gpu_full_shape.py tests/test_gpu_handle_lifecycle.py tests/test_gpu_configs0.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu > gpurun_out/t.log 2>&1; rc=$?; tail -3 gpurun_out/t.log; [ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" gpurun_out/t.log | head -20; exit 1; }
for lib in mpc-mmd_amd/libmpcmmd.so "$@"; do
  tag=$(basename $lib .so)
  MPCMMD_LIB=$lib timeout -k 10 300 python bench.py --workload mmd_opt --steps 60 --warmup 5 --cpu-seconds 0 --extra 0 > gpurun_out/ab_$tag.json || exit 1
  python -c "
import json
d=json.load(open('gpurun_out/ab_$tag.json')); print('$tag', round(d['value'],2), {k:round(v*1e3,1) for k,v in d['kernels_ms_per_step'].items()})"
done
