# Tests touching the changed kernels, the mmd_opt arms, then the cvar workload.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
bash tools/gpu_ab2.sh "$1" "tests/test_gpu_parity_mmdopt.py tests/test_gpu_full_shape.py tests/test_gpu_parity_baseline.py tests/test_gpu_free_run.py" || exit 1
timeout -k 10 120 python bench.py --cpu-seconds 0 --extra 0 --steps 100 --workload cvar > gpurun_out/ab_cvar.json 2> gpurun_out/ab_cvar.err || exit 1
python -c "import json;d=json.load(open('gpurun_out/ab_cvar.json'));print('cvar', round(d['value'],1), {k:round(v,3) for k,v in d['kernels_ms_per_step'].items()})"
