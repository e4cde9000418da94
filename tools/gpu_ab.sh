# A/B of library variants / env settings on the headline bench (no extras, no CPU baseline)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
run() {  # tag, env...
  tag=$1; shift
  env "$@" timeout -k 10 120 python bench.py --cpu-seconds 0 --extra 0 --workload ${WL:-mmd_opt} > gpurun_out/ab_$tag.json 2> gpurun_out/ab_$tag.err || return 1
  python -c "import json;d=json.load(open('gpurun_out/ab_$tag.json'));print('$tag', round(d['value'],2), {k:round(v,3) for k,v in d['kernels_ms_per_step'].items()})"
}
for spec in "$@"; do
  tag=${spec%%=*}; envs=${spec#*=}
  run $tag $envs || exit 1
done
