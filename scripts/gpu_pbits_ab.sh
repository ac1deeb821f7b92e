set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r3s2_pab; mkdir -p $OUT
B="python bench.py --steps 10 --warmup 2 --no-cpu --no-cstr --no-ntt --no-c5 --alt-bits 0"
for r in 1 2; do
  timeout -k 10 300 $B > $OUT/p51_$r.log 2>&1 || exit 1
  echo "== p51 $r"; python scripts/ab_summary.py $OUT/p51_$r.log
  timeout -k 10 300 $B --p-bits 50 --nspecial 4 > $OUT/p50_$r.log 2>&1 || exit 1
  echo "== p50 $r"; python scripts/ab_summary.py $OUT/p50_$r.log
done
