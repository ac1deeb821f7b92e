#!/bin/bash
# Same-box A/B of environment switches on one bench configuration, with the
# mul_rescale parity tests under the second setting first.
#   RUN=name BENCH_ARGS="..." bash scripts/gpu_alt_ab.sh "VAR=a" "VAR=b"
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${RUN:-alt_ab}; mkdir -p $OUT
env $2 timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu -k "mul_rescale" --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -20 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
B="python bench.py --steps 5 --warmup 1 --no-cpu --no-cstr --no-ntt --no-c5 --alt-bits 0 ${BENCH_ARGS}"
for r in 1 2; do
  i=0
  for setting in "$@"; do
    i=$((i + 1))
    env $setting timeout -k 10 300 $B > $OUT/s${i}_$r.log 2>&1 || exit 1
    echo "== $setting"; python scripts/ab_summary.py $OUT/s${i}_$r.log
  done
done
