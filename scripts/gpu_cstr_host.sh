#!/bin/bash
# CSTR (config 4) latency: host-side breakdown of the Python loop and the
# unchanged C caller's closed-loop time with / without the deferral.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${RUN:-cstr_host}
mkdir -p $OUT
timeout -k 10 200 python scripts/cstr_host_prof.py 100 > $OUT/host.log 2>&1 && cat $OUT/host.log && \
timeout -k 10 200 python scripts/cstr_c_caller.py > $OUT/c.log 2>&1 && \
timeout -k 10 200 python scripts/cstr_c_caller.py GPQHE_DEFER_GEMV=0 >> $OUT/c.log 2>&1 && \
timeout -k 10 200 python scripts/cstr_c_caller.py GPQHE_DEFER=0 >> $OUT/c.log 2>&1 && cat $OUT/c.log
