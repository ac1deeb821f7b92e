"""Per-kernel stall attribution from gpu_stall.sh passes.

  python scripts/stall_summary.py gpurun_out/<run>

SQ_WAVE_CYCLES / SQ_WAIT_* / SQ_ACTIVE_INST_* count quad-cycles per wave
(MI355X_MICROARCH.md, rocprofv3 PMC slots); the fractions below are of
SQ_WAVE_CYCLES.  WAIT_ANY = parked on s_waitcnt / barrier, WAIT_INST_ANY =
issue stall, WAIT_INST_LDS = LDS issue stall (sub-bucket of WAIT_INST_ANY).
"""
import collections
import csv
import glob
import sys

per = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(sys.argv[1] + "/p*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0].replace("void ", "")
        per[k][r["Counter_Name"]].append(float(r["Counter_Value"]))


def mean(c, n):
    v = c.get(n)
    return sum(v) / len(v) if v else float("nan")


rows = []
for k, c in per.items():
    wc = mean(c, "SQ_WAVE_CYCLES")
    if not c.get("SQ_INSTS_VALU") or mean(c, "SQ_INSTS_VALU") < 1e6:
        continue
    d = {n: mean(c, n) for n in c}
    out = [k[:44]]
    for n in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_WAIT_INST_LDS", "SQ_ACTIVE_INST_VALU",
              "SQ_ACTIVE_INST_LDS", "SQ_ACTIVE_INST_VMEM", "SQ_ACTIVE_INST_SCA", "SQ_ACTIVE_INST_MISC"):
        out.append(f"{n[3:].lower()}={d.get(n, float('nan')) / wc:.3f}")
    insts = d.get("SQ_INSTS_VALU", 0)
    out.append(f"valu={insts:.3g} lds={d.get('SQ_INSTS_LDS', 0):.3g} vmrd={d.get('SQ_INSTS_VMEM_RD', 0):.3g} "
               f"vmwr={d.get('SQ_INSTS_VMEM_WR', 0):.3g} salu={d.get('SQ_INSTS_SALU', 0):.3g}")
    if "SQ_LDS_IDX_ACTIVE" in d:
        out.append(f"lds_conflict/idx={d['SQ_LDS_BANK_CONFLICT'] / max(d['SQ_LDS_IDX_ACTIVE'], 1):.3f}")
    if "SQ_LEVEL_WAVES" in d and "SQ_WAVES" in d and "SQ_BUSY_CYCLES" in d:
        out.append(f"avg_waves={d['SQ_LEVEL_WAVES'] / max(d['SQ_BUSY_CYCLES'], 1):.1f}")
    if "SQ_INST_LEVEL_VMEM" in d:
        out.append(f"vmem_lat_q={d['SQ_INST_LEVEL_VMEM'] / max(d.get('SQ_INSTS_VMEM_RD', 0) + d.get('SQ_INSTS_VMEM_WR', 0), 1):.0f}")
    if "TCC_HIT_sum" in d and "TCC_MISS_sum" in d:
        out.append(f"l2_hit={d['TCC_HIT_sum'] / max(d['TCC_HIT_sum'] + d['TCC_MISS_sum'], 1):.3f}")
    for n in ("SQ_VMEM_TA_ADDR_FIFO_FULL", "SQ_VMEM_TA_CMD_FIFO_FULL", "SQ_LDS_DATA_FIFO_FULL"):
        if n in d:
            out.append(f"{n[3:].lower()}={d[n] / wc:.3f}")
    rows.append("\n   ".join(out))
print("\n".join(rows))
