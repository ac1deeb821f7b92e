#!/bin/bash
# Same-box A/B of the split key switch's stream arrangements (headline op):
# the default two sub-chunks (GPQHE_SPLIT_PIPE 0) and K pipelined sub-chunks
# (HBM-bound stages on the engine stream, VALU-bound ones on the second).
#   RUN=name [ROUNDS=2] [PIPES="0 2 4"] bash scripts/gpu_pipe_ab.sh
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${RUN:-pipeab}
mkdir -p $OUT
B="python bench.py --steps 10 --warmup 2 --no-cpu --no-cstr --no-ntt --no-c5 --no-gemv --alt-bits 0"
for r in $(seq 1 ${ROUNDS:-2}); do
  for p in ${PIPES:-0 2 3 4 8}; do
    GPQHE_SPLIT_PIPE=$p timeout -k 10 200 $B > $OUT/b_p${p}_r$r.log 2>&1 || { echo "bench pipe $p failed"; tail -20 $OUT/b_p${p}_r$r.log; exit 1; }
    python -c "import json,sys; d=json.loads([l for l in open('$OUT/b_p${p}_r$r.log') if l.startswith('{')][-1]); print('pipe $p round $r', round(d['value']), round(d['ms_per_step'],3))"
  done
done
