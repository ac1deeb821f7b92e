#!/bin/bash
# Default bench run, then kernel trace + PMC passes (one counter group per pass,
# no other tracing) of a short bench run and of the config 2 NTT leg.
#   RUN=name bash scripts/gpu_prof.sh
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/${RUN:-prof}
mkdir -p $OUT
if [ -z "$NO_FULL" ]; then
  timeout -k 10 600 python bench.py > $OUT/bench_full.log 2>&1 || exit 1
fi
# the kernel-trace pass runs the bench's own steps / warmup, so its mean launch
# time is the one the bench line's roofline uses; PMC passes run short
BK="python bench.py --steps 10 --warmup 2 --no-cpu --no-cstr --no-ntt --no-c5 --no-gemv --alt-bits 0 --streams 1"
B="python bench.py --steps 3 --warmup 1 --no-cpu --no-cstr --no-ntt --no-c5 --no-gemv --alt-bits 0 --streams 1"
N="python scripts/prof_ntt.py 1024"
# the gemv leg's workload (he_gemv_batch at the bench shape, 256 ciphertexts)
GV="python scripts/gemv_time.py --set bench51 --count 256 --single 0 --rot 0"
pass() {  # pass <dir> <rocprofv3 args...>  (on the bench command, the NTT leg, the gemv leg)
  d=$1; shift
  cmd=$B; [ "$d" = kt ] && cmd=$BK
  timeout -s KILL 240 rocprofv3 "$@" -d $OUT/$d -o $d --output-format csv -- $cmd > $OUT/$d.log 2>&1 || return 1
  timeout -s KILL 240 rocprofv3 "$@" -d $OUT/ntt_$d -o ntt_$d --output-format csv -- $N > $OUT/ntt_$d.log 2>&1 || return 1
  timeout -s KILL 240 rocprofv3 "$@" -d $OUT/gemv_$d -o gemv_$d --output-format csv -- $GV > $OUT/gemv_$d.log 2>&1 || return 1
}
pass kt --kernel-trace --stats || exit 1
pass fetch --pmc FETCH_SIZE || exit 1
pass write --pmc WRITE_SIZE || exit 1
pass hit --pmc TCC_HIT_sum TCC_MISS_sum || exit 1
pass sq --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_LDS SQ_BUSY_CYCLES GRBM_GUI_ACTIVE || exit 1
# the VALU instruction mix: FP64 classes (v_rndne_f64 counts in none of them), integer, conversions
pass f64 --pmc SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_CVT SQ_INSTS_VALU || exit 1
