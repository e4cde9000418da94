# cvar fused-risk profile: kernel trace + two SQ passes (GPU box)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
bash tools/prof.sh cvarf --workload cvar --extra 0 && python3 tools/pmc_table.py gpurun_out/prof_cvarf > gpurun_out/prof_cvarf/table.txt 2>&1; tail -40 gpurun_out/prof_cvarf/table.txt
