# CARLA tick A/B over library knobs (GPU box):  bash tools/carla_ab.sh N "ENV1=a ENV2=b" "ENV1=c" ...
# One bench process per setting, each with its own time limit; stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
N=$1
shift
for setting in "$@"; do
  env $setting timeout -k 10 240 python bench.py --workload carla --carla-n $N --steps 6 --warmup 1 \
    > gpurun_out/carla_ab.json 2> gpurun_out/carla_ab.err || { tail -20 gpurun_out/carla_ab.err; exit 1; }
  python -c "
import json,sys;d=json.load(open('gpurun_out/carla_ab.json'));pc=d['per_cost']
print('$setting'.ljust(40), 'mmd tick %.2f cvar tick %.2f det tick %.2f | mmd %.2f pre %.2f' % (pc['mmd_opt']['ms_per_tick'], pc['cvar']['ms_per_tick'], pc['det']['ms_per_tick'], d['ms_mmd'], d['ms_preprocess']), {k: round(v, 2) for k, v in d['kernels_ms_per_tick'].items() if v > 0.5})"
done
