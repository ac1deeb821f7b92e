#!/bin/bash
# GPU parity tests on the working tree's library, then the bench alternating
# between a baseline library (hectr_amd/lib_ab, built from another commit; delete it after the A/B: it is not gpurun-ignored)
# and the working tree's, ROUNDS times each, same box.
#   RUN=name [TESTS="tests/..."] bash scripts/gpu_libab.sh
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/${RUN:-libab}
mkdir -p $OUT
if [ -z "$NO_TESTS" ]; then
  timeout -k 10 900 python -u -m pytest ${TESTS:-tests/test_gpu_parity.py tests/test_gpu_cstr.py} -x -q -m gpu \
    --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1
  rc=$?; echo "pytest exit $rc" >> $OUT/pytest.log; [ $rc -eq 0 ] || exit 1
fi
B="python bench.py --steps 10 --warmup 2 --no-cpu --no-cstr ${LEGS:---no-ntt} --alt-bits 0 ${BENCH_ARGS}"
for r in $(seq 1 ${ROUNDS:-2}); do
  GPQHE_LIB=hectr_amd/lib_ab/libgpqhe.so timeout -k 10 300 $B > $OUT/bench_base_$r.log 2>&1 || exit 1
  timeout -k 10 300 $B > $OUT/bench_new_$r.log 2>&1 || exit 1
  # VARIANTS="name=ENVVAR=VALUE ...": the working tree's library under env switches
  for v in ${VARIANTS}; do
    env "${v#*=}" timeout -k 10 300 $B > $OUT/bench_${v%%=*}_$r.log 2>&1 || exit 1
  done
done
python scripts/ab_summary.py $OUT || true
