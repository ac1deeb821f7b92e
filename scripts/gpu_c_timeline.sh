#!/bin/bash
# Device timeline of HECTR's unchanged C harness (test-hectr cstr-hempc, 40
# steps) on the product library: rocprofv3 kernel trace, per-step kernels and
# idle gaps (scripts/cstr_timeline.py), and the harness's own timer.
#   RUN=name bash scripts/gpu_c_timeline.sh
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
ROOT=$PWD
OUT=$ROOT/gpurun_out/${RUN:-c_timeline}
mkdir -p $OUT/run/results
cd $OUT/run
LD_LIBRARY_PATH=$ROOT/hectr_amd/lib GPQHE_SEED=5 timeout -k 10 120 rocprofv3 --kernel-trace -d $OUT/tr -o tr \
  --output-format csv -- $ROOT/oracle/_ref/test-hectr cstr-hempc > $OUT/run.log 2>&1 || exit 1
cd $ROOT
python scripts/cstr_timeline.py $OUT/tr > $OUT/timeline.txt 2>&1 || exit 1
head -40 $OUT/timeline.txt
grep -E "closed-loop" $OUT/run.log
