#!/bin/bash
# Per-kernel breakdown of the other bench shapes (single-stream instrumented
# pass of bench.py): the 60-bit headline, config 5 at both prime sets, and the
# config-2 NTT kernel trace.   RUN=name bash scripts/gpu_breakdown.sh
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/${RUN:-breakdown}
mkdir -p $OUT
B="python bench.py --steps 6 --warmup 1 --no-cpu --no-cstr --no-ntt --no-c5 --alt-bits 0"
timeout -k 10 240 $B --q0-bits 60 --p-bits 60 > $OUT/bench_h60.log 2>&1 || exit 1
timeout -k 10 240 $B --logn 17 --nlimbs 12 --dnum 3 --nspecial 4 --batch 64 > $OUT/bench_c5f.log 2>&1 || exit 1
timeout -k 10 240 $B --logn 17 --nlimbs 12 --dnum 3 --nspecial 4 --batch 64 --q0-bits 60 --p-bits 60 > $OUT/bench_c5.log 2>&1 || exit 1
python scripts/ab_summary.py $OUT
RUN=${RUN:-breakdown}/ntt ROUNDS=1 bash scripts/gpu_ntt_kt.sh "X=1" || exit 1
