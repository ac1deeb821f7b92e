#!/bin/bash
# Parity, then the CSTR loop profile with the new / old whole-limb NTT.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${RUN:-small}
mkdir -p $OUT
timeout -k 10 600 python -m pytest tests/test_gpu_parity.py tests/test_gpu_cstr.py -x -q -s -m gpu > $OUT/pytest.log 2>&1 || exit 1
timeout -k 10 200 python scripts/cstr_prof.py 100 > $OUT/cstr_new.log 2>&1 || exit 1
GPQHE_NTT_WHOLE_V1=1 timeout -k 10 200 python scripts/cstr_prof.py 100 > $OUT/cstr_old.log 2>&1 || exit 1
