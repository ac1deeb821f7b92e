#!/bin/bash
# HECTR's unchanged C harness (test-hectr cstr-hempc, 40 steps, its own
# closed-loop timer) under environment settings, alternating, ROUNDS rounds:
#   RUN=name bash scripts/gpu_c_env_ab.sh "VAR=a" "VAR=b"
set -o pipefail
cd "$GRAFT_REPO_ROOT"
ROOT=$PWD
OUT=$ROOT/gpurun_out/${RUN:-c_env_ab}
mkdir -p $OUT/run/results
cd $OUT/run
for r in $(seq 1 ${ROUNDS:-5}); do
  for setting in "$@"; do
    t=$(env $setting LD_LIBRARY_PATH=$ROOT/hectr_amd/lib GPQHE_SEED=5 timeout -k 10 60 $ROOT/oracle/_ref/test-hectr cstr-hempc 2>&1 | grep -oE "closed-loop simulate\s+[0-9.]+ ms" | grep -oE "[0-9.]+ ms") || exit 1
    echo "$setting: $t"
  done
done
