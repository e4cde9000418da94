# Negative control for the beta-CEM parity tests (GPU box): build the library
# with a deliberately wrong K_red entry (csrc/k_betacem.hip: kred_perturb) and
# run the mmd_opt parity tests against it; they must FAIL.
#   bash tools/perturb_kred.sh 1   # entry 0 of every sample x 1.001  -> profiles/..._x1.001_tests.log
#   bash tools/perturb_kred.sh 2   # mantissa bit 10 of entry 0 flipped -> ..._flip_tests.log
# The build runs here (CPU container, make); the tests on the GPU box:
#   make -C mpc-mmd_amd LIB=libmpcmmd_pk1.so BUILD=build_pk1 EXTRA=-DMPCMMD_PERTURB_KRED=1 -j8
#   gpurun -- 'bash tools/perturb_kred.sh 1'
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mode=${1:-1}
lib=mpc-mmd_amd/libmpcmmd_pk$mode.so
[ -f "$lib" ] || { echo "build $lib first (see header)"; exit 2; }
mkdir -p gpurun_out
MPCMMD_LIB=$PWD/$lib timeout -k 10 600 python -u -m pytest -v --timeout 300 --timeout-method thread \
  -p no:cacheprovider tests/test_gpu_configs0.py tests/test_gpu_full_shape.py tests/test_gpu_parity_mmdopt.py \
  -m gpu > gpurun_out/perturb_kred_$mode.log 2>&1
rc=$?
grep -E "passed|failed" gpurun_out/perturb_kred_$mode.log | tail -1
# the control succeeds when the tests fail (pytest exit status 1)
[ $rc -eq 1 ] && echo "negative control OK: perturbed K_red detected" || { echo "negative control NOT detected (rc=$rc)"; exit 1; }
