"""Per-kernel PMC comparison of a scripts/gpu_pmc_ab.sh run."""
import collections
import csv
import glob
import os
import sys

run = sys.argv[1]
for vdir in sorted(glob.glob(os.path.join(run, "*/"))):
    name = os.path.basename(vdir.rstrip("/"))
    per = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in glob.glob(os.path.join(vdir, "*", "*_counter_collection.csv")):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"].split("(")[0].replace("void ", "")
            per[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
    dur = collections.defaultdict(list)
    for f in glob.glob(os.path.join(vdir, "kt", "*kernel_trace.csv")):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"].split("(")[0].replace("void ", "")
            dur[k].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    print(f"== {name}")
    rows = []
    for k, c in per.items():
        if k not in dur or sum(dur[k]) < 100:
            continue
        a = {x: sum(v) / len(v) for x, v in c.items()}
        wc = a.get("SQ_WAVE_CYCLES", 1)
        valu_busy = a.get("SQ_ACTIVE_INST_VALU", 0) * 4 / 1024 / max(a.get("GRBM_GUI_ACTIVE", 1), 1)
        rows.append((sum(dur[k]) / len(dur[k]), k, a.get("SQ_INSTS_VALU", 0) / 1e6, a.get("SQ_INSTS_LDS", 0) / 1e6,
                     a.get("SQ_WAIT_ANY", 0) / wc, a.get("SQ_WAIT_INST_ANY", 0) / wc,
                     a.get("SQ_ACTIVE_INST_ANY", 0) / wc, valu_busy))
    for us, k, valu, lds, wa, wi, ac, vb in sorted(rows, reverse=True):
        print(f"  {k:32s} {us:8.1f} us  valuInst {valu:7.1f}M  ldsInst {lds:6.2f}M  wait {wa:.2f} waitInst {wi:.2f} "
              f"active {ac:.2f}  VALUBusy~{vb:.2f}")
