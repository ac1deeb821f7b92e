#!/bin/bash
# GPU run: microbench, parity tests, bench, rocprof.  Each GPU step has its
# own time limit; a crash/abort/timeout (exit >= 2 for pytest) ends the call.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/${RUN:-r2}
mkdir -p $OUT
timeout -k 10 120 ./scripts/ubench_modmul > $OUT/ubench.log 2>&1 || { echo "ubench failed $?" >> $OUT/ubench.log; exit 1; }
timeout -k 10 900 python -m pytest tests/test_gpu_parity.py -x -q -s -m gpu > $OUT/pytest.log 2>&1
rc=$?
echo "pytest exit $rc" >> $OUT/pytest.log
[ $rc -le 1 ] || exit 1
timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu > $OUT/bench.log 2>&1 || exit 1
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/$OUT/prof" -o run -- python "$GRAFT_REPO_ROOT/bench.py" --steps 2 --warmup 1 --no-cpu > "$GRAFT_REPO_ROOT/$OUT/prof.log" 2>&1
