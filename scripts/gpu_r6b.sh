#!/bin/bash
# Round 6: every GPU test on the working tree's library, then a same-box A/B
# of the bench (headline, 60-bit, config 5, gemv legs) between the baseline
# library hectr_amd/lib_ab (HEAD before the change) and the working tree's,
# alternating ROUNDS times, then a kernel trace of the working tree's default
# bench path that must exit cleanly.      RUN=name bash scripts/gpu_r6b.sh
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/${RUN:-r6b}
mkdir -p $OUT
if [ -z "$NO_TESTS" ]; then
  timeout -k 10 1500 python -u -m pytest ${TESTS:-tests} -x -v -m gpu --timeout 900 --timeout-method thread \
    > $OUT/pytest.log 2>&1
  rc=$?; echo "pytest exit $rc" >> $OUT/pytest.log; tail -5 $OUT/pytest.log; [ $rc -eq 0 ] || exit 1
fi
B="python bench.py --steps 10 --warmup 2 --no-cpu --no-cstr --no-ntt ${BENCH_ARGS}"
for r in $(seq 1 ${ROUNDS:-2}); do
  GPQHE_LIB=hectr_amd/lib_ab/libgpqhe.so timeout -k 10 400 $B > $OUT/bench_base_$r.log 2>&1 || { echo "base bench failed"; tail -5 $OUT/bench_base_$r.log; exit 1; }
  timeout -k 10 400 $B > $OUT/bench_new_$r.log 2>&1 || { echo "new bench failed"; tail -5 $OUT/bench_new_$r.log; exit 1; }
  python scripts/ab_summary.py $OUT/bench_base_$r.log $OUT/bench_new_$r.log | grep -v "^    " || true
done
python scripts/ab_summary.py $OUT > $OUT/summary.txt || true
[ -n "$NO_TRACE" ] && exit 0
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/kt -o kt --output-format csv -- python bench.py --steps 10 --warmup 2 --no-cpu --no-cstr > $OUT/kt.log 2>&1
rc=$?; echo "rocprofv3 exit $rc" | tee -a $OUT/kt.log; [ $rc -eq 0 ] || exit 1
