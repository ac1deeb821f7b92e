#!/bin/bash
# Round 6: the small-N / rotation / teardown GPU tests on the working tree's
# library, then a same-box A/B of the bench (every leg but the CPU baseline
# and the NTT roundtrip) between hectr_amd/lib_ab and the working tree's,
# alternating ROUNDS times, then a kernel trace of the default bench path
# that must exit cleanly.      RUN=name bash scripts/gpu_r6d.sh
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/${RUN:-r6d}
mkdir -p $OUT
if [ -z "$NO_TESTS" ]; then
  timeout -k 10 1200 python -u -m pytest ${TESTS:-tests/test_gpu_hectr_caller.py tests/test_gpu_cstr.py tests/test_gpu_parity.py tests/test_gpu_rotations.py tests/test_gpu_teardown.py} \
    ${KSEL:+-k "$KSEL"} -x -v -m gpu --timeout 600 --timeout-method thread > $OUT/pytest.log 2>&1
  rc=$?; echo "pytest exit $rc" >> $OUT/pytest.log; tail -4 $OUT/pytest.log; [ $rc -eq 0 ] || exit 1
fi
B="python bench.py --steps 10 --warmup 2 --no-cpu --no-ntt ${BENCH_ARGS}"
for r in $(seq 1 ${ROUNDS:-2}); do
  GPQHE_LIB=hectr_amd/lib_ab/libgpqhe.so timeout -k 10 400 $B > $OUT/bench_base_$r.log 2>&1 || { echo "base bench failed"; tail -5 $OUT/bench_base_$r.log; exit 1; }
  timeout -k 10 400 $B > $OUT/bench_new_$r.log 2>&1 || { echo "new bench failed"; tail -5 $OUT/bench_new_$r.log; exit 1; }
  python scripts/ab_summary.py $OUT/bench_base_$r.log $OUT/bench_new_$r.log | grep -v "^    " || true
done
python scripts/ab_summary.py $OUT > $OUT/summary.txt || true
if [ -z "$NO_TRACE" ]; then
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/kt -o kt --output-format csv -- python bench.py --steps 10 --warmup 2 --no-cpu --no-cstr > $OUT/kt.log 2>&1
rc=$?; echo "rocprofv3 exit $rc" | tee -a $OUT/kt.log; [ $rc -eq 0 ] || exit 1
fi
# the C harness with and without the speculated gemvs (same library)
[ -n "$SPEC_AB" ] || exit 0
for r in $(seq 1 ${SPEC_ROUNDS:-2}); do
  for v in 1 0; do
    GPQHE_SPEC_GEMV=$v timeout -k 10 200 python -c "
import sys; sys.path.insert(0, '.'); import bench, json
print('spec_gemv=$v', json.dumps({k: v for k, v in bench.cstr_c_caller(reps=5).items() if k != 'config4_c_driver'}))
" >> $OUT/spec_ab.txt 2>&1 || exit 1
  done
done
cat $OUT/spec_ab.txt | cut -c1-200
