#!/bin/bash
# Config 2 group-size sweep (GPQHE_NTT_GROUP_MIB, api.cpp ntt_batch): the
# roundtrip of 1024 polys per size (and per environment setting in ENVS),
# alternating, twice (plus EXTRA_ROUNDS).
#   RUN=name [SIZES="96 128 160 192 224"] [ENVS="GPQHE_NTT_REV=0 GPQHE_NTT_REV=1"] bash scripts/gpu_ntt_group.sh
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/${RUN:-nttgrp}
mkdir -p $OUT
for r in 1 2 ${EXTRA_ROUNDS}; do
  for m in ${SIZES:-96 128 160 192 224}; do
    for e in ${ENVS:-X=0}; do
      tag=g${m}_${e//=/}_$r
      env $e GPQHE_NTT_GROUP_MIB=$m timeout -k 10 240 python scripts/prof_ntt.py > $OUT/$tag.json 2> $OUT/$tag.err || { cat $OUT/$tag.err; exit 1; }
      echo "$m MiB $e: $(python -c "import json;print(round(json.load(open('$OUT/$tag.json'))['roundtrip_ms'],3))") ms"
    done
  done
done
