#!/bin/bash
# Round 6: same-box A/B of libraries on the headline + gemv legs (no CSTR /
# NTT / config 5 / CPU legs): LIBS="name=path ..." alternating ROUNDS times;
# optional parity tests first (TESTS).      RUN=name bash scripts/gpu_r6g.sh
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/${RUN:-r6g}
mkdir -p $OUT
if [ -n "$TESTS" ]; then
  timeout -k 10 1200 python -u -m pytest $TESTS ${KSEL:+-k "$KSEL"} -x -v -m gpu --timeout 600 --timeout-method thread \
    > $OUT/pytest.log 2>&1
  rc=$?; echo "pytest exit $rc" >> $OUT/pytest.log; tail -4 $OUT/pytest.log; [ $rc -eq 0 ] || exit 1
fi
NO_NTT=--no-ntt; [ -n "$NTT" ] && NO_NTT=""
B="python bench.py --steps 10 --warmup 2 --no-cpu --no-cstr $NO_NTT ${BENCH_ARGS}"
for r in $(seq 1 ${ROUNDS:-2}); do
  for v in ${LIBS:-new=hectr_amd/lib/libgpqhe.so}; do
    GPQHE_LIB=${v#*=} timeout -k 10 400 $B > $OUT/bench_${v%%=*}_$r.log 2>&1 || { echo "bench $v failed"; tail -5 $OUT/bench_${v%%=*}_$r.log; exit 1; }
    python scripts/ab_summary.py $OUT/bench_${v%%=*}_$r.log | grep -v "^    " || true
  done
done
python scripts/ab_summary.py $OUT > $OUT/summary.txt || true
