#!/bin/bash
# Round 6, first GPU session: the new parity / teardown / 8-rank tests, the
# default bench line, and a rocprofv3 kernel trace of the default bench path
# that must exit cleanly.    RUN=name bash scripts/gpu_r6a.sh
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/${RUN:-r6a}
mkdir -p $OUT
timeout -k 10 1500 python -u -m pytest ${TESTS:-tests/test_gpu_gemv_shapes.py tests/test_gpu_teardown.py tests/test_gpu_dist.py} \
  -x -v -m gpu --timeout 900 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; echo "pytest exit $rc" >> $OUT/pytest.log; tail -25 $OUT/pytest.log; [ $rc -eq 0 ] || exit 1
[ -n "$NO_BENCH" ] && exit 0
timeout -k 10 400 python bench.py > $OUT/bench.log 2>&1 || { echo "bench failed"; tail -20 $OUT/bench.log; exit 1; }
tail -c 600 $OUT/bench.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/kt -o kt --output-format csv -- python bench.py --steps 10 --warmup 2 --no-cpu --no-cstr > $OUT/kt.log 2>&1
rc=$?; echo "rocprofv3 exit $rc" | tee -a $OUT/kt.log; [ $rc -eq 0 ] || exit 1
