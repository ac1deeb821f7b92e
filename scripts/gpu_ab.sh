#!/bin/bash
# GPU parity tests, then the bench once per variant.  VARIANTS is a
# space-separated list of NAME=ENVVAR=VALUE items ("base" runs unmodified).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/${RUN:-ab}
mkdir -p $OUT
timeout -k 10 900 python -m pytest tests/test_gpu_parity.py tests/test_gpu_cstr.py -x -q -s -m gpu > $OUT/pytest.log 2>&1
rc=$?; echo "pytest exit $rc" >> $OUT/pytest.log; [ $rc -eq 0 ] || exit 1
for v in base ${VARIANTS}; do
  name=${v%%=*}; kv=${v#*=}
  if [ "$v" = base ]; then
    timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu --no-cstr --ntt-polys 256 ${BENCH_ARGS} > $OUT/bench_base.log 2>&1 || exit 1
  else
    env "$kv" timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu --no-cstr --ntt-polys 256 ${BENCH_ARGS} > $OUT/bench_$name.log 2>&1 || exit 1
  fi
done
