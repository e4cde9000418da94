# k_bqp LDS-conflict attribution.  Build (container):
#   bash tools/qp_variants.sh build      -> mpc-mmd_amd/libmpcmmd_qpV.so, V = 1 (no cost phase),
#                                           2 (staging + row loads), 3 (staging only)
# Measure (GPU box): bash tools/qp_variants.sh run   -> gpurun_out/qpv/*.csv + a table
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
if [ "$1" = build ]; then
  for v in 1 2 3; do
    make -C mpc-mmd_amd -j8 LIB=libmpcmmd_qp$v.so BUILD=build_qp$v EXTRA=-DMPCMMD_QP_VARIANT=$v > /dev/null || exit 1
  done
  exit 0
fi
export TMPDIR=/tmp
mkdir -p gpurun_out/qpv
ARGS="--steps 4 --warmup 1 --profile-steps 2 --cpu-seconds 0 --extra 0"
for v in 0 1 2 3; do
  lib=mpc-mmd_amd/libmpcmmd.so
  [ $v -gt 0 ] && lib=mpc-mmd_amd/libmpcmmd_qp$v.so
  MPCMMD_LIB=$lib MPCMMD_GROUPS=1 timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_WAVES SQ_WAVE_CYCLES \
    -d gpurun_out/qpv/v$v -o run --output-format csv -- python3 bench.py $ARGS > gpurun_out/qpv/v$v.log 2>&1 || { tail -5 gpurun_out/qpv/v$v.log; exit 1; }
  MPCMMD_LIB=$lib MPCMMD_GROUPS=1 timeout -s KILL 120 rocprofv3 --kernel-trace --stats -d gpurun_out/qpv/kt$v -o run --output-format csv -- python3 bench.py $ARGS > gpurun_out/qpv/kt$v.log 2>&1 || { tail -5 gpurun_out/qpv/kt$v.log; exit 1; }
done
python3 - <<'PY'
import csv, glob
for v in range(4):
    f = glob.glob(f"gpurun_out/qpv/v{v}/**/*counter_collection.csv", recursive=True)
    tot = {}
    n = 0
    for r in csv.DictReader(open(f[0])):
        if "k_bqp" not in r["Kernel_Name"]:
            continue
        tot[r["Counter_Name"]] = tot.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    k = glob.glob(f"gpurun_out/qpv/kt{v}/**/*kernel_stats.csv", recursive=True)
    us = [float(r["AverageNs"]) / 1e3 for r in csv.DictReader(open(k[0])) if "k_bqp" in r["Name"]]
    disp = {0: "full", 1: "no cost phase", 2: "staging + row loads", 3: "staging only"}[v]
    lds, cf = tot.get("SQ_INSTS_LDS", 0), tot.get("SQ_LDS_BANK_CONFLICT", 0)
    print(f"v{v} {disp:20s} k_bqp {us[0] if us else float('nan'):6.1f} us  INSTS_LDS {lds:.3g}  BANK_CONFLICT {cf:.3g} "
          f"({cf / max(lds, 1):.2f} per LDS instr)  WAIT_INST_LDS {tot.get('SQ_WAIT_INST_LDS', 0):.3g}  VALU {tot.get('SQ_INSTS_VALU', 0):.3g}")
PY
