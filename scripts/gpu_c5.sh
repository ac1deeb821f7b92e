#!/bin/bash
# Parity, then config 5 (N=2^17, L=12, dnum=3) on the fused path vs the generic one.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${RUN:-c5}
mkdir -p $OUT
timeout -k 10 900 python -m pytest tests/test_gpu_parity.py tests/test_gpu_cstr.py -x -q -s -m gpu > $OUT/pytest.log 2>&1 || exit 1
B="timeout -k 10 300 python bench.py --logn 17 --nlimbs 12 --dnum 3 --batch 64 --steps 3 --warmup 1 --no-cpu --no-cstr --no-ntt --alt-bits 0"
$B > $OUT/bench_c5.log 2>&1 || exit 1
GPQHE_NTT_V1=1 $B > $OUT/bench_c5_generic.log 2>&1 || exit 1
$B --q0-bits 60 --p-bits 60 > $OUT/bench_c5_p60.log 2>&1 || exit 1
