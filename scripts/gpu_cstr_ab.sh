#!/bin/bash
# GPU tests touching the small-N path, smoke, then the CSTR loop (config 4)
# on the baseline library (hectr_amd/lib_ab) and the working tree's,
# alternating; HECTR's C harness on both.   RUN=name bash scripts/gpu_cstr_ab.sh
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${RUN:-cstr_ab}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -x -v -m gpu --timeout 120 --timeout-method thread ${TESTS:-} > $OUT/pytest.log 2>&1 || { echo "pytest failed"; grep -E "FAIL|Error|error" $OUT/pytest.log | head -20; tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" || exit 1
for r in 1 2; do
  GPQHE_LIB=hectr_amd/lib_ab/libgpqhe.so timeout -k 10 200 python scripts/cstr_prof.py 100 > $OUT/base_$r.log 2>&1 || exit 1
  timeout -k 10 200 python scripts/cstr_prof.py 100 > $OUT/new_$r.log 2>&1 || exit 1
  head -1 $OUT/base_$r.log $OUT/new_$r.log
done
cat $OUT/new_2.log
timeout -k 10 200 python scripts/cstr_c_caller.py > $OUT/c.log 2>&1 && cat $OUT/c.log
