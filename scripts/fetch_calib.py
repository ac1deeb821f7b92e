"""FETCH_SIZE / WRITE_SIZE calibration per access pattern: every kernel of
scripts/ubench_mem.hip reads 1 GiB and writes 1 GiB per launch.

    python scripts/fetch_calib.py gpurun_out/<run>   (dirs fcal_fetch, fcal_write)

Prints measured / true bytes for each kernel (FETCH_SIZE, WRITE_SIZE in KiB)."""
import collections
import csv
import os
import sys

TRUE = 1 << 30
run = sys.argv[1]
vals = collections.defaultdict(dict)
for d, c in (("fcal_fetch", "FETCH_SIZE"), ("fcal_write", "WRITE_SIZE")):
    per = collections.defaultdict(list)
    for r in csv.DictReader(open(os.path.join(run, d, d + "_counter_collection.csv"))):
        per[r["Kernel_Name"].split("(")[0].replace("void ", "")].append(float(r["Counter_Value"]))
    for k, v in per.items():
        vals[k][c] = sorted(v)[len(v) // 2] * 1024  # median over launches
print(f"{'kernel':10s} {'FETCH/true':>10s} {'WRITE/true':>10s}")
for k, e in vals.items():
    print(f"{k:10s} {e.get('FETCH_SIZE', 0) / TRUE:10.3f} {e.get('WRITE_SIZE', 0) / TRUE:10.3f}")
