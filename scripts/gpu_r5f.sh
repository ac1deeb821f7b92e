#!/bin/bash
# Round-5 headline iteration: parity tests of the ct x ct path on the working
# tree's library, then same-box A/B against lib_var/* (gpu_var_ab.sh).
#   RUN=name [TESTS_K=...] [ROUNDS=3] bash scripts/gpu_r5f.sh
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/${RUN:-r5f}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu -k "${TESTS_K:-mul or streams or relin}" --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 || { echo "pytest failed"; tail -40 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
RUN=${RUN:-r5f}/ab ROUNDS=${ROUNDS:-3} LEGS="${LEGS:---no-ntt --no-c5 --no-gemv}" ALT=${ALT:-0} bash scripts/gpu_var_ab.sh
