# default bench (all workloads) for each library given
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
for lib in "$@"; do
  tag=$(basename $lib .so)
  MPCMMD_LIB=$lib timeout -k 10 500 python bench.py --cpu-seconds 0 > gpurun_out/full_$tag.json || exit 1
  python -c "
import json
d=json.load(open('gpurun_out/full_$tag.json')); x=d['extra_workloads']
print('$tag', round(d['value'],2), {k:round(v.get('value',0),2) for k,v in x.items()}, round(d['roofline']['avg_us'],1))"
done
