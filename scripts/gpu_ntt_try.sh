#!/bin/bash
# NTT parity (-k ntt) under each environment setting, then per-kernel config-2
# times under each (scripts/gpu_ntt_kt.sh):  RUN=name bash scripts/gpu_ntt_try.sh "VAR=a" ...
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/${RUN:-ntt_try}
mkdir -p $OUT
for setting in "$@"; do
  env $setting timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu -k ntt --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { echo "pytest failed ($setting)"; tail -30 $OUT/pytest.log; exit 1; }
  echo "$setting: $(tail -1 $OUT/pytest.log)"
done
RUN=${RUN:-ntt_try} bash scripts/gpu_ntt_kt.sh "$@"
