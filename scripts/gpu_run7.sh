#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/${RUN:-r7}
mkdir -p $OUT
timeout -k 10 900 python -m pytest tests/test_gpu_parity.py tests/test_gpu_cstr.py -x -q -s -m gpu > $OUT/pytest.log 2>&1
rc=$?; echo "pytest exit $rc" >> $OUT/pytest.log; [ $rc -le 1 ] || exit 1
timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu --no-cstr > $OUT/bench.log 2>&1 || exit 1
GPQHE_UNFUSED=1 timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu --no-cstr > $OUT/bench_unfused.log 2>&1 || exit 1
