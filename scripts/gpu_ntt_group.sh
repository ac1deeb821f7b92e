#!/bin/bash
# Config 2 group-size sweep (GPQHE_NTT_GROUP_MIB, api.cpp ntt_batch): the
# roundtrip of 1024 polys per size, twice each, alternating.
#   RUN=name [SIZES="96 128 160 192 224"] bash scripts/gpu_ntt_group.sh
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/${RUN:-nttgrp}
mkdir -p $OUT
for r in 1 2; do
  for m in ${SIZES:-96 128 160 192 224}; do
    GPQHE_NTT_GROUP_MIB=$m timeout -k 10 240 python scripts/prof_ntt.py > $OUT/g${m}_$r.json 2> $OUT/g${m}_$r.err || { cat $OUT/g${m}_$r.err; exit 1; }
    echo "$m MiB: $(python -c "import json;print(round(json.load(open('$OUT/g${m}_$r.json'))['roundtrip_ms'],3))") ms"
  done
done
