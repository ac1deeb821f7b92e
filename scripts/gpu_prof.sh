#!/bin/bash
# Default bench run, then kernel trace + PMC passes (one counter group per pass,
# no other tracing) of a short bench run.  RUN=name bash scripts/gpu_prof.sh
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/${RUN:-prof}
mkdir -p $OUT
if [ -z "$NO_FULL" ]; then
  timeout -k 10 600 python bench.py > $OUT/bench_full.log 2>&1 || exit 1
fi
B="python bench.py --steps 3 --warmup 1 --no-cpu --no-cstr --no-ntt --alt-bits 0"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/kt -o kt --output-format csv -- $B > $OUT/kt.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d $OUT/fetch -o fetch --output-format csv -- $B > $OUT/fetch.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d $OUT/write -o write --output-format csv -- $B > $OUT/write.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum -d $OUT/hit -o hit --output-format csv -- $B > $OUT/hit.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS -d $OUT/sq -o sq --output-format csv -- $B > $OUT/sq.log 2>&1 || exit 1
