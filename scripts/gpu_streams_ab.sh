#!/bin/bash
# Headline with the batch on one HIP stream vs two sub-chunks on two streams,
# alternating, same box.   RUN=name [ROUNDS=3] bash scripts/gpu_streams_ab.sh
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/${RUN:-streams_ab}
mkdir -p $OUT
B="python bench.py --steps 10 --warmup 2 --no-cpu --no-cstr --no-ntt --no-c5 ${ALT:---alt-bits 0}"
for r in $(seq 1 ${ROUNDS:-3}); do
  for s in 1 2; do
    timeout -k 10 240 $B --streams $s > $OUT/bench_s${s}_$r.log 2>&1 || exit 1
    python - $OUT/bench_s${s}_$r.log $s <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith('{"metric"')][-1])
print(f"streams {sys.argv[2]}: {d['value']:.0f} ct-mult/s  60-bit {d.get('value_60bit', 0):.0f}  ms/step {d['ms_per_step']:.3f}")
PY
  done
done
