#!/bin/bash
# Round 6: the small-N GPU tests on the working tree's library, then HECTR's
# C harness and the config-4 C driver alternating an environment switch
# (AB_VAR, values 1 / 0), then the C harness's device timeline.
#   RUN=name AB_VAR=GPQHE_SPEC_MODUP_SPLIT bash scripts/gpu_r6k.sh
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/${RUN:-r6k}
mkdir -p $OUT
if [ -z "$NO_TESTS" ]; then
  timeout -k 10 900 python -u -m pytest ${TESTS:-tests/test_gpu_hectr_caller.py tests/test_gpu_cstr.py tests/test_gpu_parity.py} \
    ${KSEL:+-k "$KSEL"} -x -v -m gpu --timeout 600 --timeout-method thread > $OUT/pytest.log 2>&1
  rc=$?; echo "pytest exit $rc" >> $OUT/pytest.log; tail -4 $OUT/pytest.log; [ $rc -eq 0 ] || exit 1
fi
V=${AB_VAR:-GPQHE_SPEC_MODUP_SPLIT}
for r in $(seq 1 ${ROUNDS:-3}); do
  for v in 1 0; do
    # AB_VAR=GPQHE_LIB: 1 = the working tree's library, 0 = hectr_amd/lib_ab's
    if [ "$V" = GPQHE_LIB ]; then E="GPQHE_LIB=$([ $v = 1 ] && echo hectr_amd/lib || echo hectr_amd/lib_ab)/libgpqhe.so"; else E="$V=$v"; fi
    env $E timeout -k 10 200 python -c "
import sys; sys.path.insert(0, '.'); import bench, json
d = bench.cstr_c_caller(reps=5)
c4 = d.get('config4_c_driver', {})
print('$V=$v', json.dumps({k: v for k, v in d.items() if k != 'config4_c_driver'}), 'c4', c4.get('steps_per_s'))
" >> $OUT/ab.txt 2>&1 || { tail -20 $OUT/ab.txt; exit 1; }
  done
done
cut -c1-260 $OUT/ab.txt
[ -n "$NO_TL" ] && exit 0
RUN=${RUN:-r6k}/tl1 bash scripts/gpu_c_timeline.sh > /dev/null || exit 1
head -12 $OUT/tl1/timeline.txt
