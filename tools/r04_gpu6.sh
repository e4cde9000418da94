# A/B of k_roll_cand variants (cvar workload, kernel times)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
for lib in mpc-mmd_amd/libmpcmmd.so "$@"; do
  tag=$(basename $lib .so)
  MPCMMD_LIB=$lib timeout -k 10 200 python bench.py --workload cvar --steps 100 --warmup 10 --cpu-seconds 0 --extra 0 > gpurun_out/ab_$tag.json || exit 1
  python -c "
import json
d=json.load(open('gpurun_out/ab_$tag.json')); print('$tag', round(d['value'],1), {k:round(v*1e3,1) for k,v in d['kernels_ms_per_step'].items()})"
done
