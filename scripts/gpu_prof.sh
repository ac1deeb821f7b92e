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
B="python bench.py --steps 3 --warmup 1 --no-cpu --no-cstr --no-ntt --no-c5 --alt-bits 0"
N="python scripts/prof_ntt.py 1024"
pass() {  # pass <dir> <rocprofv3 args...>  (on the bench command, then on the NTT leg)
  d=$1; shift
  timeout -s KILL 240 rocprofv3 "$@" -d $OUT/$d -o $d --output-format csv -- $B > $OUT/$d.log 2>&1 || return 1
  timeout -s KILL 240 rocprofv3 "$@" -d $OUT/ntt_$d -o ntt_$d --output-format csv -- $N > $OUT/ntt_$d.log 2>&1 || return 1
}
pass kt --kernel-trace --stats || exit 1
pass fetch --pmc FETCH_SIZE || exit 1
pass write --pmc WRITE_SIZE || exit 1
pass hit --pmc TCC_HIT_sum TCC_MISS_sum || exit 1
pass sq --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_LDS SQ_BUSY_CYCLES GRBM_GUI_ACTIVE || exit 1
