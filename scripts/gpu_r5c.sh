#!/bin/bash
# Round-5 stream-arrangement A/B (split key switch pipelined over K sub-chunks
# on the engine + second stream) with kernel traces for the overlap.
#   RUN=name bash scripts/gpu_r5c.sh
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/${RUN:-r5c}
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu -k "streams or bench_shape" --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1 || { echo "pytest failed"; tail -40 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
RUN=${RUN:-r5c}/pipe ROUNDS=${ROUNDS:-2} PIPES="${PIPES:-0 2 3 4}" bash scripts/gpu_pipe_ab.sh || exit 1
B="python bench.py --steps 10 --warmup 2 --no-cpu --no-cstr --no-ntt --no-c5 --no-gemv --alt-bits 0"
for p in ${KT_PIPES:-2 4}; do
  GPQHE_SPLIT_PIPE=$p timeout -s KILL 240 rocprofv3 --kernel-trace --stats -d $OUT/kt_pipe$p -o kt_pipe$p --output-format csv -- $B > $OUT/kt_pipe$p.log 2>&1 || exit 1
done
