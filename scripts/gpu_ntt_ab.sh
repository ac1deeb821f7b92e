#!/bin/bash
# NTT parity under each environment setting, then the config-2 roundtrip leg
# under each (same box, alternating):  RUN=name bash scripts/gpu_ntt_ab.sh "VAR=a" "VAR=b"
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${RUN:-ntt_ab}
mkdir -p $OUT
for setting in "$@"; do
  env $setting timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu -k "ntt or mul_rescale" --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { echo "pytest failed ($setting)"; tail -30 $OUT/pytest.log; exit 1; }
  echo "$setting: $(tail -1 $OUT/pytest.log)"
done
for r in 1 2; do
  i=0
  for setting in "$@"; do
    i=$((i + 1))
    env $setting timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu --no-cstr --no-c5 --alt-bits 0 > $OUT/bench_${i}_$r.log 2>&1 || { echo "bench failed ($setting)"; tail -30 $OUT/bench_${i}_$r.log; exit 1; }
    echo "== $setting round $r"; python scripts/ab_summary.py $OUT/bench_${i}_$r.log | grep -i "ntt\|ct-mult"
  done
done
