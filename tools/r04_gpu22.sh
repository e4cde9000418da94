# round artifacts: smoke, every GPU test, default bench, rocprof stats + PMC (mmd_opt and cvar)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
bash tools/gpu.sh round r04f && \
bash tools/prof.sh r04f_cvar --workload cvar --extra 0 && \
python3 tools/pmc_table.py gpurun_out/prof_r04f > gpurun_out/prof_r04f/table.txt 2>&1 && \
python3 tools/pmc_table.py gpurun_out/prof_r04f_cvar > gpurun_out/prof_r04f_cvar/table.txt 2>&1 && echo ALLDONE
