#!/bin/bash
# Config-5 iteration run: the GPU parity tests named by TESTS_K on the working
# tree's library, then the config-5 same-box A/B (scripts/gpu_c5ab.sh).
#   RUN=name TESTS_K="c5" [C5_60=1] bash scripts/gpu_c5r.sh
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/${RUN:-c5r}
mkdir -p $OUT
if [ -n "$TESTS_K" ]; then
  timeout -k 10 ${TEST_LIMIT:-600} python -u -m pytest tests/test_gpu_parity.py -k "$TESTS_K" -x -v --timeout 300 \
    --timeout-method thread > $OUT/pytest.log 2>&1
  rc=$?
  echo "pytest rc $rc" >> $OUT/pytest.log
  tail -3 $OUT/pytest.log
  [ $rc -eq 0 ] || exit 1
fi
RUN=${RUN:-c5r}/ab bash scripts/gpu_c5ab.sh
