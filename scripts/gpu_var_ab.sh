#!/bin/bash
# Same-box A/B of variant libraries (scripts/build_variant.sh) against the
# working tree's library, alternating, ROUNDS times each:
#   RUN=name [ROUNDS=2] [LEGS="--no-ntt"] [VARS="a b"] bash scripts/gpu_var_ab.sh
# Each bench run is the headline op (default streams) plus the instrumented
# single-stream pass that gives per-kernel times.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/${RUN:-varab}
mkdir -p $OUT
VARS=${VARS:-$(ls hectr_amd/lib_var 2>/dev/null)}
B="python bench.py --steps ${STEPS:-10} --warmup 2 --no-cpu --no-cstr ${LEGS:---no-ntt --no-c5} --alt-bits ${ALT:-0} ${BENCH_ARGS}"
for r in $(seq 1 ${ROUNDS:-2}); do
  timeout -k 10 300 $B > $OUT/bench_base_$r.log 2>&1 || { echo "base bench failed"; tail -20 $OUT/bench_base_$r.log; exit 1; }
  for v in $VARS; do
    GPQHE_LIB=hectr_amd/lib_var/$v/libgpqhe.so timeout -k 10 300 $B > $OUT/bench_${v}_$r.log 2>&1 || { echo "bench $v failed"; tail -20 $OUT/bench_${v}_$r.log; exit 1; }
  done
done
python scripts/ab_summary.py $OUT || true
