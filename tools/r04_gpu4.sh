set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity_baseline.py tests/test_gpu_free_run.py tests/test_gpu_full_shape.py tests/test_gpu_sweep_concurrent.py tests/test_validation_golden.py tests/test_gpu_carla.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu > gpurun_out/gpu_risk.log 2>&1; rc=$?; tail -3 gpurun_out/gpu_risk.log; [ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" gpurun_out/gpu_risk.log | head -20; exit 1; }
MPCMMD_RISK_FUSED=0 timeout -k 10 300 python bench.py --workload cvar --steps 200 --warmup 20 --cpu-seconds 0 --extra 0 > gpurun_out/bench_cvar_rows.json && \
timeout -k 10 300 python bench.py --workload cvar --steps 200 --warmup 20 --cpu-seconds 0 --extra 0 > gpurun_out/bench_cvar_cand.json && \
python -c "
import json
for f in ('rows','cand'):
    d=json.load(open('gpurun_out/bench_cvar_%s.json'%f)); print(f, round(d['value'],1), {k:round(v*1e3,1) for k,v in d['kernels_ms_per_step'].items()})"
