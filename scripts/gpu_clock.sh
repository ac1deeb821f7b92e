#!/bin/bash
# Effective shader clock per kernel: GRBM_GUI_ACTIVE / 8 XCDs / kernel time
# (MI355X_MICROARCH.md, DVFS give-back).  RUN=name bash scripts/gpu_clock.sh
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/${RUN:-clock}
mkdir -p $OUT
B="python bench.py --steps 3 --warmup 1 --no-cpu --no-cstr --no-ntt --alt-bits 0"
timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT -d $OUT/clk -o clk --output-format csv -- $B > $OUT/clk.log 2>&1 || exit 1
python - $OUT/clk/clk_counter_collection.csv <<'PY'
import csv, collections, sys
acc = collections.defaultdict(lambda: [0, 0.0, 0.0])
for r in csv.DictReader(open(sys.argv[1])):
    if r["Counter_Name"] != "GRBM_GUI_ACTIVE":
        continue
    k = r["Kernel_Name"].split("(")[0][:40]
    dt = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
    a = acc[k]; a[0] += 1; a[1] += float(r["Counter_Value"]); a[2] += dt
for k, (n, c, t) in sorted(acc.items(), key=lambda kv: -kv[1][2]):
    if n >= 10:
        print(f"{k:40s} n={n:4d} {t / n * 1e6:8.1f} us  clock {c / 8 / t / 1e9:.2f} GHz")
PY
