#!/bin/bash
# Config-4 device timeline (kernels + copies per control step, idle gaps) and
# the host-side breakdown of the same loop.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/${RUN:-cstr_timeline}
mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace -d $OUT/tl -o tl --output-format csv -- python scripts/cstr_prof.py 100 noprof > $OUT/run.log 2>&1 || exit 1
python scripts/cstr_timeline.py $OUT/tl > $OUT/timeline.txt 2>&1; head -80 $OUT/timeline.txt
timeout -k 10 200 python scripts/cstr_host_prof.py 100 > $OUT/host.log 2>&1 && cat $OUT/host.log && \
timeout -k 10 200 python scripts/cstr_c_caller.py > $OUT/c.log 2>&1 && cat $OUT/c.log
