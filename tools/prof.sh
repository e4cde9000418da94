# rocprofv3 passes over a short bench run (GPU box).  Usage:
#   bash tools/prof.sh TAG [bench args...]
# Writes gpurun_out/prof_TAG/{stats,pmc1..pmc4}.  One counter group per pass
# (rocprofv3 does not split counters over passes); every pass has its own
# time limit and the chain stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
TAG=${1:-run}
shift
ARGS="--steps 4 --warmup 1 --profile-steps 2 --cpu-seconds 0 $*"
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
timeout -s KILL 240 rocprofv3 --kernel-trace --stats -d $OUT/stats -o run --output-format csv -- python3 bench.py $ARGS > $OUT/stats.log 2>&1 && \
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU -d $OUT/pmc1 -o run --output-format csv -- python3 bench.py $ARGS > $OUT/pmc1.log 2>&1 && \
timeout -s KILL 240 rocprofv3 --pmc SQ_INSTS_LDS SQ_INSTS_SMEM SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR -d $OUT/pmc2 -o run --output-format csv -- python3 bench.py $ARGS > $OUT/pmc2.log 2>&1 && \
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE -d $OUT/pmc3 -o run --output-format csv -- python3 bench.py $ARGS > $OUT/pmc3.log 2>&1 && \
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE TCC_HIT_sum TCC_MISS_sum -d $OUT/pmc4 -o run --output-format csv -- python3 bench.py $ARGS > $OUT/pmc4.log 2>&1
