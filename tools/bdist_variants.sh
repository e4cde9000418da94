# k_bdist timing builds (results are garbage; GPU box): the default library,
# then MPCMMD_BDIST_VARIANT=1 (no mirror phase) and =2 (no stores at all),
# k_bdist ms per configs[1] step from bench.py's per-kernel times.
#   build first:  make -C mpc-mmd_amd LIB=libmpcmmd_bd1.so BUILD=build_bd1 EXTRA=-DMPCMMD_BDIST_VARIANT=1 (and 2)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
for lib in mpc-mmd_amd/libmpcmmd.so mpc-mmd_amd/libmpcmmd_bd1.so mpc-mmd_amd/libmpcmmd_bd2.so; do
  MPCMMD_LIB=$lib timeout -k 10 300 python bench.py --steps 6 --warmup 2 --extra 0 --cpu-seconds 0 > gpurun_out/bd.json 2> gpurun_out/bd.err || { tail -5 gpurun_out/bd.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/bd.json')); print('$lib', 'bdist ms/step', round(d['kernels_ms_per_step']['bdist'], 3))"
done
