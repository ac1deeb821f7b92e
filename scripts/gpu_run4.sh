#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/${RUN:-r4}
mkdir -p $OUT
timeout -k 10 900 python -m pytest tests/test_gpu_cstr.py tests/test_gpu_parity.py -x -q -s -m gpu > $OUT/pytest.log 2>&1
rc=$?; echo "pytest exit $rc" >> $OUT/pytest.log; [ $rc -le 1 ] || exit 1
for d in 8 4 2; do
  timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu --no-cstr --dnum $d > $OUT/bench_d$d.log 2>&1 || exit 1
done
timeout -k 10 300 python bench.py --steps 5 --warmup 2 --dnum 2 > $OUT/bench_full.log 2>&1 || exit 1
