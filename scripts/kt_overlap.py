"""Kernel concurrency from a rocprofv3 kernel trace (--kernel-trace, csv).

python scripts/kt_overlap.py <run dir> [name filter]
For the kernels whose names contain the filter (default: the split key
switch's five), prints the summed kernel time, the union of their intervals
(device busy), the time with two or more of them running at once and how that
overlapped time splits by kernel pair.
"""
import csv
import glob
import os
import sys
from collections import defaultdict

KEYS = ("ksq_kernel", "ks_colsf", "dn_colsf", "d2_rows", "ks_cols4", "dn_cols")


def short(name):
    n = name.split("(")[0].replace("void ", "")
    if n.startswith("ksq_kernel"):
        return "ksq<keep>" if ", true," in n else "ksq<drop>"
    return n.split("<")[0]


def main():
    d = sys.argv[1]
    filt = sys.argv[2:] or KEYS
    f = sorted(glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True))[0]
    iv = []
    with open(f) as fh:
        for r in csv.DictReader(fh):
            name = r["Kernel_Name"]
            if any(k in name for k in filt):
                iv.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(name)))
    iv.sort()
    total = sum(e - s for s, e, _ in iv)
    # sweep: busy (>= 1 running) and overlapped (>= 2) time, overlap by pair
    ev = sorted([(s, 1, i) for i, (s, e, _) in enumerate(iv)] + [(e, -1, i) for i, (s, e, _) in enumerate(iv)])
    run, busy, over, last = set(), 0, 0, None
    pair = defaultdict(int)
    for t, kind, i in ev:
        if last is not None and run:
            busy += t - last
            if len(run) >= 2:
                over += t - last
                names = sorted({iv[j][2] for j in run})
                pair[" + ".join(names)] += t - last
        last = t
        (run.add if kind == 1 else run.discard)(i)
    print(f"{f}: {len(iv)} launches, kernel time {total / 1e6:.2f} ms, busy {busy / 1e6:.2f} ms, "
          f">= 2 running {over / 1e6:.2f} ms ({100 * over / max(busy, 1):.1f} % of busy)")
    per = defaultdict(lambda: [0, 0])
    for s, e, n in iv:
        per[n][0] += 1
        per[n][1] += e - s
    for n, (c, t) in sorted(per.items(), key=lambda kv: -kv[1][1]):
        print(f"   {n:16s} {c:4d} x {t / c / 1e3:8.1f} us")
    for k, v in sorted(pair.items(), key=lambda kv: -kv[1]):
        print(f"   overlap {k:40s} {v / 1e6:.3f} ms")


if __name__ == "__main__":
    main()
