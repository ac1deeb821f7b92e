#!/bin/bash
# Config 5 (n=2^17, L=12, dnum 3, K 4, 64 pairs) same-box A/B of the
# working tree's library against hectr_amd/lib_var/*, at the headline's prime
# sizes (and the 60-bit ones with C5_60=1), per-kernel times.
#   RUN=name [ROUNDS=2] bash scripts/gpu_c5ab.sh
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/${RUN:-c5ab}
mkdir -p $OUT
B="python bench.py --steps 6 --warmup 1 --no-cpu --no-cstr --no-ntt --no-c5 --alt-bits 0 --logn 17 --nlimbs 12 --dnum 3 --nspecial 4 --batch 64"
for r in $(seq 1 ${ROUNDS:-2}); do
  timeout -k 10 240 $B > $OUT/bench_base_$r.log 2>&1 || exit 1
  [ -n "$C5_60" ] && { timeout -k 10 240 $B --q0-bits 60 --p-bits 60 > $OUT/bench_base60_$r.log 2>&1 || exit 1; }
  for v in $(ls hectr_amd/lib_var 2>/dev/null); do
    GPQHE_LIB=hectr_amd/lib_var/$v/libgpqhe.so timeout -k 10 240 $B > $OUT/bench_${v}_$r.log 2>&1 || exit 1
    [ -n "$C5_60" ] && { GPQHE_LIB=hectr_amd/lib_var/$v/libgpqhe.so timeout -k 10 240 $B --q0-bits 60 --p-bits 60 > $OUT/bench_${v}60_$r.log 2>&1 || exit 1; }
  done
done
python scripts/ab_summary.py $OUT
