#!/bin/bash
# Round 6: gemv / rotation parity on the working tree's library, then the
# gemv timing script alternating an environment switch (AB_VAR 1 / 0) on
# three shapes (bench51 and bench_d2 at 256 ciphertexts, c5f at 64).
#   RUN=name AB_VAR=GPQHE_DN_PRE bash scripts/gpu_r6m.sh
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/${RUN:-r6m}
mkdir -p $OUT
if [ -z "$NO_TESTS" ]; then
  timeout -k 10 900 python -u -m pytest ${TESTS:-tests/test_gpu_rotations.py tests/test_gpu_gemv_shapes.py} \
    ${KSEL:+-k "$KSEL"} -x -v -m gpu --timeout 600 --timeout-method thread > $OUT/pytest.log 2>&1
  rc=$?; echo "pytest exit $rc" >> $OUT/pytest.log; tail -4 $OUT/pytest.log; [ $rc -eq 0 ] || exit 1
fi
V=${AB_VAR:-GPQHE_DN_PRE}
for r in $(seq 1 ${ROUNDS:-2}); do
  for v in 1 0; do
    for cfg in "bench51 256" "bench_d2 256" "c5f 64"; do
      set -- $cfg
      echo -n "$V=$v $1 $2 " >> $OUT/ab.txt
      env $V=$v timeout -k 10 300 python scripts/gemv_time.py --set $1 --count $2 --single 0 --rot 1 --reps 5 >> $OUT/ab.txt 2>$OUT/err.log || { cat $OUT/err.log; exit 1; }
    done
  done
done
cut -c1-220 $OUT/ab.txt
