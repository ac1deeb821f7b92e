#!/bin/bash
# Round-4 iteration run: the GPU tests named by TESTS_K (pytest -k) on the
# working tree's library, then the same-box A/B of hectr_amd/lib_var/* against
# it (scripts/gpu_var_ab.sh), then the stall PMC passes (scripts/gpu_stall.sh)
# unless NO_STALL is set.  Every GPU step has its own time limit and a failing
# step ends the run.
#   RUN=name TESTS_K="mul or ntt" bash scripts/gpu_r4a.sh
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/${RUN:-r4a}
mkdir -p $OUT
if [ -n "$TESTS_K" ]; then
  timeout -k 10 ${TEST_LIMIT:-600} python -u -m pytest ${TEST_FILES:-tests/test_gpu_parity.py tests/test_gpu_dist.py} \
    -k "$TESTS_K" -x -v --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1
  rc=$?
  echo "pytest rc $rc" >> $OUT/pytest.log
  tail -3 $OUT/pytest.log
  [ $rc -eq 0 ] || exit 1
fi
if [ -d hectr_amd/lib_var ] && [ -z "$NO_AB" ]; then
  RUN=${RUN:-r4a}/ab bash scripts/gpu_var_ab.sh || exit 1
fi
if [ -z "$NO_STALL" ]; then
  RUN=${RUN:-r4a}/stall bash scripts/gpu_stall.sh || exit 1
fi
