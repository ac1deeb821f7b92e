#!/bin/bash
# Round-5 CU-mask A/B of the split key switch's stream arrangements (the
# GPQHE_SPLIT_PIPE / GPQHE_S2_MASK experiment in api.cpp), headline only, same
# box, two alternating rounds; then one kernel trace per masked arrangement
# for scripts/kt_overlap.py.    RUN=name bash scripts/gpu_r5m.sh
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/${RUN:-r5m}
mkdir -p $OUT
B="python bench.py --no-cpu --no-cstr --no-ntt --no-c5 --no-gemv --alt-bits 0"
VARS="0:0 2:0 2:8 2:16 4:8 0:8"
for r in 1 2; do
  for v in $VARS; do
    p=${v%:*}; m=${v#*:}
    GPQHE_SPLIT_PIPE=$p GPQHE_S2_MASK=$m timeout -k 10 300 $B > $OUT/b_p${p}_m${m}_$r.log 2>&1 || { echo "bench $v failed"; tail -5 $OUT/b_p${p}_m${m}_$r.log; exit 1; }
    python -c "import json; l=[x for x in open('$OUT/b_p${p}_m${m}_$r.log') if x.startswith('{')][-1]; d=json.loads(l); print('pipe $p mask $m round $r %.0f %.3f' % (d['value'], d['ms_per_step']))"
  done
done
for v in 2:8 0:8; do
  p=${v%:*}; m=${v#*:}
  GPQHE_SPLIT_PIPE=$p GPQHE_S2_MASK=$m timeout -s KILL 240 rocprofv3 --kernel-trace -d $OUT/kt_p${p}_m${m} -o kt --output-format csv -- python bench.py --steps 5 --warmup 1 --no-cpu --no-cstr --no-ntt --no-c5 --no-gemv --alt-bits 0 > $OUT/kt_p${p}_m${m}.log 2>&1 || { echo "trace $v failed"; exit 1; }
  python scripts/kt_overlap.py $OUT/kt_p${p}_m${m} | head -30
done
