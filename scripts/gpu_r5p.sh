#!/bin/bash
# Round-5 A/Bs: (1) parity of the m60 set (60-bit q0, special primes below
# 2^51, three digits), then the headline op on that set against the 60-bit
# q0 / P set (dnum 2) and the all-FP64 set at dnum 3, same box, alternating;
# (2) gemv_time.py on the working tree's library and each lib_var/* variant.
#   RUN=name [SETS="bench51"] bash scripts/gpu_r5p.sh
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/${RUN:-r5p}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_rotations.py -x -v -m gpu -k "${TESTS_K:-m60}" --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 || { echo "pytest failed"; tail -40 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
B="python bench.py --no-cpu --no-cstr --no-ntt --no-c5 --no-gemv --alt-bits 0"
for r in 1 2; do
  for v in "60 60 2" "60 51 3" "51 51 3" "51 51 2"; do
    set -- $v
    timeout -k 10 300 $B --q0-bits $1 --p-bits $2 --dnum $3 > $OUT/b_${1}_${2}_${3}_$r.log 2>&1 || { echo "bench $v failed"; tail -5 $OUT/b_${1}_${2}_${3}_$r.log; exit 1; }
    python -c "import json; l=[x for x in open('$OUT/b_${1}_${2}_${3}_$r.log') if x.startswith('{')][-1]; d=json.loads(l); print('q0 $1 P $2 dnum $3 r$r: %.0f ct-mult/s  %s' % (d['value'], d['config']['workload'][-60:]))"
  done
done
for r in 1 2; do
  for set in ${SETS:-bench51}; do
    for v in base $(ls hectr_amd/lib_var 2>/dev/null); do
      L=hectr_amd/lib/libgpqhe.so; [ $v != base ] && L=hectr_amd/lib_var/$v/libgpqhe.so
      GPQHE_LIB=$L timeout -k 10 300 python scripts/gemv_time.py --set $set --count ${COUNT:-64} --single 0 > $OUT/t_${set}_${v}_$r.json 2>&1 || { echo "$v failed"; tail -5 $OUT/t_${set}_${v}_$r.json; exit 1; }
      python -c "import json; d=json.loads(open('$OUT/t_${set}_${v}_$r.json').read().strip().splitlines()[-1]); k=d['gemv_batch_kernels_us_per_ct']; print('$set $v r$r gemv %.2f us  inner %.2f  c0 %.2f  rot %.2f' % (d['gemv_batch_us_per_ct'], k.get('gemv_win_kernel', 0), k.get('gemv_c0_kernel', 0), d['rot_batch_us_per_ct']))"
    done
  done
done
