# cvar A/B of library variants (30 steps)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity_baseline.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu -k "beta_planes or lockstep" > gpurun_out/t.log 2>&1; rc=$?; tail -2 gpurun_out/t.log; [ $rc -eq 0 ] || exit 1
for lib in mpc-mmd_amd/libmpcmmd.so "$@"; do
  tag=$(basename $lib .so)
  MPCMMD_LIB=$lib timeout -k 10 200 python bench.py --workload cvar --steps 100 --warmup 10 --cpu-seconds 0 --extra 0 > gpurun_out/ab_$tag.json || exit 1
  python -c "
import json
d=json.load(open('gpurun_out/ab_$tag.json')); print('$tag', round(d['value'],1), {k:round(v*1e3,1) for k,v in d['kernels_ms_per_step'].items()})"
done
