#!/bin/bash
# GPU parity tests, then the same short bench under each environment setting
# given (same box, back to back):  RUN=name bash scripts/gpu_ab.sh "VAR=a" "VAR=b" ...
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/${RUN:-ab}
mkdir -p $OUT
if [ -z "$NO_TESTS" ]; then
  timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread ${TESTS:-} > $OUT/pytest.log 2>&1 || { echo "pytest failed"; tail -40 $OUT/pytest.log; exit 1; }
  tail -2 $OUT/pytest.log
fi
i=0
for setting in "$@"; do
  i=$((i + 1))
  env $setting timeout -k 10 300 python bench.py --no-cpu --no-cstr ${BENCH_ARGS:-} > $OUT/bench_$i.log 2>&1 || { echo "bench failed ($setting)"; tail -30 $OUT/bench_$i.log; exit 1; }
  echo "== $setting"
  python scripts/ab_summary.py $OUT/bench_$i.log
done
