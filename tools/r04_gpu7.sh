# parity of both risk paths, then the A/B (rows default vs MPCMMD_RISK_FUSED=1)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity_baseline.py tests/test_gpu_free_run.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -m gpu > gpurun_out/t.log 2>&1; rc=$?; tail -3 gpurun_out/t.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 200 python bench.py --workload cvar --steps 100 --warmup 10 --cpu-seconds 0 --extra 0 > gpurun_out/ab_rows.json && MPCMMD_LIB=mpc-mmd_amd/libmpcmmd_bp32.so timeout -k 10 200 python bench.py --workload cvar --steps 100 --warmup 10 --cpu-seconds 0 --extra 0 > gpurun_out/ab_bp32.json && \
MPCMMD_RISK_FUSED=1 timeout -k 10 200 python bench.py --workload cvar --steps 100 --warmup 10 --cpu-seconds 0 --extra 0 > gpurun_out/ab_fused.json && \
python -c "
import json
for f in ('rows','bp32','fused'):
    d=json.load(open('gpurun_out/ab_%s.json'%f)); print(f, round(d['value'],1), {k:round(v*1e3,1) for k,v in d['kernels_ms_per_step'].items()})"
