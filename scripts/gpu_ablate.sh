#!/bin/bash
# Timing-only ablation runs of the bench (results are wrong when GPQHE_ABLATE != 0).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${RUN:-abl}
mkdir -p $OUT
for a in ${MASKS:-0 1 2 4 8 3 15}; do
  GPQHE_ABLATE=$a timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu --no-cstr --no-ntt > $OUT/bench_a$a.log 2>&1 || exit 1
done
