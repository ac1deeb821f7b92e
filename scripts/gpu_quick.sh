#!/bin/bash
# Parity tests then a bench run without the CPU baseline (iteration loop).
#   RUN=name bash scripts/gpu_quick.sh [extra bench args]
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/${RUN:-quick}
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 || { echo "pytest failed"; tail -40 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
timeout -k 10 600 python bench.py --no-cpu "$@" > $OUT/bench.log 2>&1 || { echo "bench failed"; tail -30 $OUT/bench.log; exit 1; }
python - $OUT/bench.log <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
print("value", round(d["value"]), "alt", round(d.get("alt_primes", {}).get("value", 0)), "cstr", d.get("cstr", {}).get("steps_per_s"))
for k, v in d["kernels"].items():
    print(f"  {k:28s} {v['avg_us']:8.1f} us {v['streamed_GBs']:8.0f} GB/s")
PY
