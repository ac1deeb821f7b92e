#!/bin/bash
# Parity, then the CSTR loop with batched vs per-diagonal he_gemv launches.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${RUN:-gemv}
mkdir -p $OUT
timeout -k 10 600 python -m pytest tests/test_gpu_parity.py tests/test_gpu_cstr.py -x -q -s -m gpu > $OUT/pytest.log 2>&1 || exit 1
B="timeout -k 10 300 python bench.py --steps 2 --warmup 1 --no-cpu --no-ntt --alt-bits 0"
$B > $OUT/bench_base.log 2>&1 || exit 1
GPQHE_GEMV_PER_DIAG=1 $B > $OUT/bench_perdiag.log 2>&1 || exit 1
