#!/bin/bash
# Sub-chunk sweep of the headline op (Infinity-Cache-resident
# intermediates): GPQHE_CHUNK pairs per chunk, working-tree library (streaming
# stores for y / T1 / accd / conv) against hectr_amd/lib_ab (built with
# -DGPQHE_PLAIN_STORES), same box, alternating.
#   RUN=name CHUNKS="256 64 16 8" bash scripts/gpu_chunk_sweep.sh
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/${RUN:-sweep}
mkdir -p $OUT
B="python bench.py --steps 10 --warmup 2 --no-cpu --no-cstr --no-ntt --no-c5 --alt-bits 0"
for r in $(seq 1 ${ROUNDS:-1}); do
  for c in ${CHUNKS:-256 128 64 32 16 8}; do
    GPQHE_CHUNK=$c timeout -k 10 300 $B > $OUT/bench_nt_c${c}_$r.log 2>&1 || exit 1
    GPQHE_CHUNK=$c GPQHE_LIB=hectr_amd/lib_ab/libgpqhe.so timeout -k 10 300 $B > $OUT/bench_plain_c${c}_$r.log 2>&1 || exit 1
    echo "chunk $c round $r done"
  done
done
python scripts/ab_summary.py $OUT || true
