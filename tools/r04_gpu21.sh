# k_front distributed GEMVs: bit comparison with the base build, cvar A/B
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 300 python tools/ab_bits.py mpc-mmd_amd/libmpcmmd_base.so mpc-mmd_amd/libmpcmmd.so cvar mmd_opt || exit 1
bash tools/r04_gpu14.sh mpc-mmd_amd/libmpcmmd_base.so
