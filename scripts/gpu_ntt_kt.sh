#!/bin/bash
# Per-kernel config-2 times under environment settings (rocprofv3 kernel trace
# of scripts/prof_ntt.py, one run per setting, same box, ROUNDS rounds):
#   RUN=name bash scripts/gpu_ntt_kt.sh "VAR=a" "VAR=b"
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/${RUN:-ntt_kt}
mkdir -p $OUT
for r in $(seq 1 ${ROUNDS:-2}); do
  i=0
  for setting in "$@"; do
    i=$((i + 1))
    d=kt_${i}_$r
    env $setting timeout -s KILL 180 rocprofv3 --kernel-trace --stats -d $OUT/$d -o $d --output-format csv -- python scripts/prof_ntt.py 1024 > $OUT/$d.log 2>&1 || { echo "failed ($setting)"; tail -20 $OUT/$d.log; exit 1; }
    echo "== $setting round $r: $(grep -o '"roundtrip_ms": [0-9.]*' $OUT/$d.log)"
    python - $OUT/$d/${d}_kernel_stats.csv <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if "ntt" in r["Name"]:
        print(f'   {r["Name"][:60]:60s} n={r["Calls"]:>4s} avg {float(r["AverageNs"])/1e3:8.1f} us')
PY
  done
done
