#!/bin/bash
# Round-5 gemv inner-kernel iteration: rotation parity tests on the working
# tree's library, then gemv_time.py on it and on each lib_var/* variant
# (same box, alternating).
#   RUN=name [SETS="bench51"] [COUNT=64] bash scripts/gpu_r5d.sh
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/${RUN:-r5d}
mkdir -p $OUT
if [ -z "$NO_TESTS" ]; then
  timeout -k 10 900 python -u -m pytest tests/test_gpu_rotations.py -x -v -m gpu -k "${TESTS_K:-bench51 or bench_d2 or c14}" --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 || { echo "pytest failed"; tail -40 $OUT/pytest.log; exit 1; }
  tail -1 $OUT/pytest.log
fi
for r in 1 2; do
  for set in ${SETS:-bench51}; do
    for v in base $(ls hectr_amd/lib_var 2>/dev/null); do
      L=hectr_amd/lib/libgpqhe.so; [ $v != base ] && L=hectr_amd/lib_var/$v/libgpqhe.so
      GPQHE_LIB=$L timeout -k 10 300 python scripts/gemv_time.py --set $set --count ${COUNT:-64} --single 0 > $OUT/t_${set}_${v}_$r.json 2>&1 || { echo "$v failed"; tail -5 $OUT/t_${set}_${v}_$r.json; exit 1; }
      python -c "import json; d=json.loads(open('$OUT/t_${set}_${v}_$r.json').read().strip().splitlines()[-1]); k=d['gemv_batch_kernels_us_per_ct']; print('$set $v r$r gemv %.2f us  inner %.2f  c0 %.2f  rot %.2f' % (d['gemv_batch_us_per_ct'], k.get('gemv_win_kernel', 0), k.get('gemv_c0_kernel', 0), d['rot_batch_us_per_ct']))"
    done
  done
done
