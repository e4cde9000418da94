# bench.py A/B over environment settings (GPU box):
#   bash tools/bench_ab.sh "WORKLOAD STEPS" "ENV=a ..." "ENV=b ..."   (each setting twice, interleaved)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
read -r WL STEPS <<< "$1"
shift
for rep in 1 2; do
  for setting in "$@"; do
    env $setting timeout -k 10 300 python bench.py --workload $WL --steps $STEPS --warmup 3 --extra 0 --cpu-seconds 0 \
      > gpurun_out/bench_ab.json 2> gpurun_out/bench_ab.err || { tail -20 gpurun_out/bench_ab.err; exit 1; }
    python -c "
import json;d=json.load(open('gpurun_out/bench_ab.json'))
print('$setting'.ljust(60), '$WL %.2f steps/s median %.3f ms' % (d['value'], d['median_ms_per_step']))"
  done
done
