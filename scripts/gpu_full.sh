#!/bin/bash
# GPU tests, smoke, then the default bench + rocprof kernel trace + PMC passes.
#   RUN=name bash scripts/gpu_full.sh
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/${RUN:-full}
mkdir -p $OUT
timeout -k 10 1000 python -u -m pytest tests -x -v -m gpu --timeout 600 --timeout-method thread > $OUT/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $OUT/pytest.log; exit 1; }
tail -3 $OUT/pytest.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo "smoke failed"; cat $OUT/smoke.log; exit 1; }
cat $OUT/smoke.log
RUN=${RUN:-full} bash scripts/gpu_prof.sh || exit 1
tail -c 3000 $OUT/bench_full.log
if [ -n "$FCAL" ]; then
  # FETCH_SIZE / WRITE_SIZE calibration per access pattern (scripts/fetch_calib.py)
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $OUT/fcal_fetch -o fcal_fetch --output-format csv -- ./scripts/ubench_mem > $OUT/fcal_fetch.log 2>&1 || exit 1
  timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $OUT/fcal_write -o fcal_write --output-format csv -- ./scripts/ubench_mem > $OUT/fcal_write.log 2>&1 || exit 1
  python scripts/fetch_calib.py $OUT > $OUT/fcal.txt 2>&1; cat $OUT/fcal.txt
fi
