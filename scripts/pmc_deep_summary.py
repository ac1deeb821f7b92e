"""Per-kernel means of every counter in gpurun_out/<run>/p*/p*_counter_collection.csv."""
import collections
import csv
import glob
import sys

per = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(sys.argv[1] + "/p*/p*_counter_collection.csv"):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0].replace("void ", "")[:34]
        per[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, c in per.items():
    if len(c.get("SQ_INSTS_VALU", [])) < 10:
        continue
    print(k)
    print("   " + "  ".join(f"{n[3:]}={sum(v) / len(v):.3g}" for n, v in sorted(c.items())))
