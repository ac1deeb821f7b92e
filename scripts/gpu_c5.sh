#!/bin/bash
# Config 5 at both prime-size sets: its parity cases, then the bench's config5
# leg (headline primes and the 60-bit set) with the other legs skipped.
#   RUN=name bash scripts/gpu_c5.sh
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/${RUN:-c5}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -v -m gpu -k "c5" --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 || { echo "pytest failed"; tail -40 $OUT/pytest.log; exit 1; }
tail -3 $OUT/pytest.log
timeout -k 10 300 python bench.py --no-cpu --no-cstr --no-ntt > $OUT/bench.log 2>&1 || { echo "bench failed"; tail -30 $OUT/bench.log; exit 1; }
python - $OUT/bench.log <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
c5 = d["config5"]
print("headline", round(d["value"]), "60-bit", round(d.get("value_60bit", 0)))
print("config5", round(c5["value"]), c5["workload"], "| 60-bit", round(c5.get("value_60bit", 0)), "frac", round(c5["op_roofline_frac"], 3))
PY
