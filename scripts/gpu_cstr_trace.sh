#!/bin/bash
# Kernel trace of the encrypted CSTR loop (config 4): per-kernel device time per step.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/${RUN:-cstr_trace}
mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/kt -o kt --output-format csv -- python scripts/cstr_prof.py 100 noprof > $OUT/run.log 2>&1 || exit 1
head -3 $OUT/run.log
python - $OUT/kt/kt_kernel_stats.csv <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:14]:
    print(f'{r["Name"][:50]:50s} calls={int(r["Calls"]):6d} avg={float(r["AverageNs"])/1e3:7.2f} us total={float(r["TotalDurationNs"])/1e6:8.2f} ms')
PY
