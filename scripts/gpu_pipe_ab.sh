#!/bin/bash
# Same-box A/B of the split key switch's stream arrangements (headline op):
# the default two sub-chunks, and GPQHE_SPLIT_PIPE / GPQHE_SPLIT_HCU variants.
#   RUN=name [ROUNDS=2] bash scripts/gpu_pipe_ab.sh
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${RUN:-pipeab}
mkdir -p $OUT
B="python bench.py --steps 10 --warmup 2 --no-cpu --no-cstr --no-ntt --no-c5 --no-gemv --alt-bits 0"
for r in $(seq 1 ${ROUNDS:-2}); do
  for v in "0 0" "2 0" "4 0" "4 8" "4 12" "8 0"; do
    set -- $v
    GPQHE_SPLIT_PIPE=$1 GPQHE_SPLIT_HCU=$2 timeout -k 10 200 $B > $OUT/b_p$1_h$2_r$r.log 2>&1 || { echo "bench $v failed"; tail -20 $OUT/b_p$1_h$2_r$r.log; exit 1; }
    python -c "import json,sys; d=json.loads([l for l in open('$OUT/b_p$1_h$2_r$r.log') if l.startswith('{')][-1]); print('pipe $1 hcu $2 round $r', round(d['value']), round(d['ms_per_step'],3))"
  done
done
