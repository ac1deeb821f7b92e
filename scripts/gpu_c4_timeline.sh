#!/bin/bash
# Device timeline of config 4 at its own shape (harness/cstr_run.c: the
# reference's unchanged hectr_simulate, N = 100, 32 slots) on the product
# library: rocprofv3 kernel trace, per-step kernels and gaps, and the
# closed-loop time the reference's own timer prints.   RUN=name bash scripts/gpu_c4_timeline.sh
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
ROOT=$PWD
OUT=$ROOT/gpurun_out/${RUN:-c4_timeline}
mkdir -p $OUT
LD_LIBRARY_PATH=$ROOT/hectr_amd/lib GPQHE_SEED=5 timeout -k 10 60 $ROOT/oracle/_ref/cstr-run hempc 100 $OUT/t.bin > $OUT/plain.log 2>&1 || exit 1
grep -E "closed-loop" $OUT/plain.log
LD_LIBRARY_PATH=$ROOT/hectr_amd/lib GPQHE_SEED=5 timeout -k 10 120 rocprofv3 --kernel-trace -d $OUT/tr -o tr \
  --output-format csv -- $ROOT/oracle/_ref/cstr-run hempc 100 $OUT/t2.bin > $OUT/run.log 2>&1 || exit 1
python scripts/cstr_timeline.py $OUT/tr > $OUT/timeline.txt 2>&1 || exit 1
head -20 $OUT/timeline.txt
GPQHE_HOSTPROF=1 LD_LIBRARY_PATH=$ROOT/hectr_amd/lib GPQHE_SEED=5 timeout -k 10 60 $ROOT/oracle/_ref/cstr-run hempc 100 $OUT/t3.bin > $OUT/hp.log 2>&1 || exit 1
grep -E "hostprof" $OUT/hp.log | head -20
