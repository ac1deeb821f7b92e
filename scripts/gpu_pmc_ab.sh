#!/bin/bash
# PMC counters of a short bench run, once per variant (VARIANTS as gpu_ab.sh).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/${RUN:-pmcab}
mkdir -p $OUT
B="python bench.py --steps 2 --warmup 1 --no-cpu --no-cstr --no-ntt"
for v in base ${VARIANTS}; do
  name=${v%%=*}; kv=${v#*=}
  [ "$v" = base ] && kv="GPQHE_BASE=1"
  env "$kv" timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS -d $OUT/$name/sq -o sq --output-format csv -- $B > $OUT/$name.sq.log 2>&1 || exit 1
  env "$kv" timeout -k 10 300 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU GRBM_GUI_ACTIVE SQ_BUSY_CYCLES -d $OUT/$name/valu -o valu --output-format csv -- $B > $OUT/$name.valu.log 2>&1 || exit 1
  env "$kv" timeout -k 10 300 rocprofv3 --kernel-trace -d $OUT/$name/kt -o kt --output-format csv -- $B > $OUT/$name.kt.log 2>&1 || exit 1
done
