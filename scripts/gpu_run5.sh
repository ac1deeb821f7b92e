#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/${RUN:-r5}
mkdir -p $OUT
timeout -k 10 900 python -m pytest tests/test_gpu_parity.py tests/test_gpu_cstr.py -x -q -s -m gpu > $OUT/pytest.log 2>&1
rc=$?; echo "pytest exit $rc" >> $OUT/pytest.log; [ $rc -le 1 ] || exit 1
timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu --no-cstr > $OUT/bench.log 2>&1 || exit 1
GPQHE_NTT_V1=1 timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu --no-cstr > $OUT/bench_v1.log 2>&1 || exit 1
