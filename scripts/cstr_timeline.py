"""Device timeline of the encrypted CSTR loop (config 4) from a rocprofv3
kernel + memory-copy trace: per control step the kernels and copies issued,
the busy time, and the idle gaps between them (steps end at the D2H copy of
he_dcd).  Usage: python scripts/cstr_timeline.py <dir with *_kernel_trace.csv>"""
import csv
import glob
import os
import sys

import numpy as np

d = sys.argv[1]


def load(pattern):
    f = glob.glob(os.path.join(d, "**", pattern), recursive=True)
    return list(csv.DictReader(open(f[0]))) if f else []


ev = []
for r in load("*kernel_trace.csv"):
    ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "K", r["Kernel_Name"].split("(")[0][:40]))
for r in load("*memory_copy_trace.csv"):
    ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "C", r.get("Direction", r.get("Operation", "copy"))))
ev.sort()
print("files:", [os.path.relpath(f, d) for f in glob.glob(os.path.join(d, "**", "*.csv"), recursive=True)])
print("copy kinds:", sorted({e[3] for e in ev if e[2] == "C"}))
ends = [i for i, e in enumerate(ev) if e[2] == "C" and "DEVICE_TO_HOST" in e[3].upper()]
if len(ends) < 4:  # no D2H copy: the decoder's kernel ends each step
    ends = [i for i, e in enumerate(ev) if e[2] == "K" and ("fft_dec" in e[3] or "inv_dcd" in e[3])]
steps = []
for a, b in zip(ends[:-1], ends[1:]):
    seg = ev[a + 1:b + 1]
    span = seg[-1][1] - ev[a][1]
    # busy = union of the intervals (kernels of the side stream overlap)
    busy, cur0, cur1 = 0, None, None
    for e0, e1, *_ in sorted(seg):
        if cur1 is None or e0 > cur1:
            busy += (cur1 - cur0) if cur1 is not None else 0
            cur0, cur1 = e0, e1
        else:
            cur1 = max(cur1, e1)
    busy += (cur1 - cur0) if cur1 is not None else 0
    steps.append((span, busy, sum(e[2] == "K" for e in seg), sum(e[2] == "C" for e in seg), seg))
steps = steps[len(steps) // 2:]  # steady state: the second half
span = np.median([s[0] for s in steps]) / 1e3
busy = np.median([s[1] for s in steps]) / 1e3
print(f"{len(steps)} steps: span {span:.1f} us/step (D2H end to D2H end), device busy {busy:.1f} us (union), "
      f"kernels {np.median([s[2] for s in steps]):.0f}, copies {np.median([s[3] for s in steps]):.0f}")
seg = steps[len(steps) // 2][4]
t0 = seg[0][0]
prev = None
for e in seg:
    gap = (e[0] - prev) / 1e3 if prev else 0.0
    print(f"  +{(e[0] - t0) / 1e3:8.1f} us  gap {gap:6.1f}  dur {(e[1] - e[0]) / 1e3:6.1f}  {e[2]} {e[3]}")
    prev = e[1]
