# round artifacts: smoke, every GPU test, default bench, rocprof stats + PMC (mmd_opt and cvar)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
bash tools/gpu.sh round r04d && \
bash tools/prof.sh r04d_cvar --workload cvar --extra 0 && \
python3 tools/pmc_table.py gpurun_out/prof_r04d > gpurun_out/prof_r04d/table.txt 2>&1 && \
python3 tools/pmc_table.py gpurun_out/prof_r04d_cvar > gpurun_out/prof_r04d_cvar/table.txt 2>&1 && echo ALLDONE
