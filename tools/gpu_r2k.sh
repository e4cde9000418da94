# Candidate library (MPCMMD_LIB=$1): beta-noise tests and the cvar bench
# against the default library, then the torchrun launch path at N = 1.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
CAND=${1:-mpc-mmd_amd/libmpcmmd.so}
MPCMMD_LIB=$CAND timeout -k 10 400 python -u -m pytest tests/test_gpu_parity_baseline.py tests/test_gpu_full_shape.py tests/test_gpu_free_run.py -x -v --timeout 240 --timeout-method thread -p no:cacheprovider > gpurun_out/k_tests.log 2>&1 || { tail -30 gpurun_out/k_tests.log; exit 1; }
grep -E "passed|failed" gpurun_out/k_tests.log | tail -1
for lib in mpc-mmd_amd/libmpcmmd.so $CAND; do
  MPCMMD_LIB=$lib timeout -k 10 120 python bench.py --cpu-seconds 0 --extra 0 --workload cvar > gpurun_out/k_cvar.json 2> gpurun_out/k_cvar.err || exit 1
  python -c "import json;d=json.load(open('gpurun_out/k_cvar.json'));print('$lib cvar', round(d['value'],1), {k:round(v,3) for k,v in d['kernels_ms_per_step'].items()})"
done
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 1 --steps 40 --warmup 5 --cpu-seconds 0 --extra 0 > gpurun_out/k_trun.json 2> gpurun_out/k_trun.err || exit 1
python -c "import json;d=json.load(open('gpurun_out/k_trun.json'));print('torchrun N=1', round(d['value'],2), d['n_gpus'], d['config']['parallelism'])"
