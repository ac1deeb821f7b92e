#!/bin/bash
# Same-box A/B: FP64 basis conversion on/off (51-bit primes) and the 60-bit set.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${RUN:-r27}
mkdir -p $OUT
timeout -k 10 600 python -m pytest tests/test_gpu_parity.py -x -q -s -m gpu -k "bench51 or bench_d2" > $OUT/pytest.log 2>&1 || exit 1
B="timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu --no-cstr --no-ntt --alt-bits 0"
$B > $OUT/bench_fb.log 2>&1 || exit 1
GPQHE_NO_F64FBC=1 $B > $OUT/bench_nofb.log 2>&1 || exit 1
$B --p-bits 60 --q0-bits 60 > $OUT/bench_p60.log 2>&1 || exit 1
$B > $OUT/bench_fb2.log 2>&1 || exit 1
