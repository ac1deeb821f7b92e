#!/bin/bash
# Rehearsal of the driver's N>1 bench launch on a one-GPU box: 2 ranks share
# cuda:0 over gloo (RCCL needs distinct devices); checks the JSON line and the
# aggregate value.  Never launch N=8 here.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${RUN:-dist}
mkdir -p $OUT
HECTR_DIST_BACKEND=gloo timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29531 bench.py --gpus 2 --steps 3 --warmup 1 --batch 64 --no-cpu \
  --cstr-steps 20 > $OUT/bench_n2.log 2>&1 || exit 1
