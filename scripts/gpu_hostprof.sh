#!/bin/bash
# Host time of HECTR's unchanged C harness (test-hectr cstr-hempc, 40 steps)
# per library entry point and one steady-state step's call timeline
# (GPQHE_HOSTPROF=2, printed by hectx_exit).   RUN=name bash scripts/gpu_hostprof.sh
set -o pipefail
cd "$GRAFT_REPO_ROOT"
ROOT=$PWD
OUT=$ROOT/gpurun_out/${RUN:-hostprof}
mkdir -p $OUT/run/results
cd $OUT/run
for r in 1 2; do
  LD_LIBRARY_PATH=$ROOT/hectr_amd/lib GPQHE_HOSTPROF=2 ${HP_ENV} timeout -k 10 120 $ROOT/oracle/_ref/test-hectr cstr-hempc > $OUT/hp_$r.log 2>&1 || exit 1
done
grep -E "closed-loop|hostprof" $OUT/hp_2.log
# the config-4 C driver (100 steps, 32 slots) the same way
if [ -n "$C4" ]; then
  LD_LIBRARY_PATH=$ROOT/hectr_amd/lib GPQHE_SEED=5 GPQHE_HOSTPROF=2 timeout -k 10 120 $ROOT/oracle/_ref/cstr-run hempc 100 $OUT/run/c4.bin > $OUT/hp_c4.log 2>&1 || exit 1
  grep -E "closed-loop|hostprof" $OUT/hp_c4.log
fi
