#!/usr/bin/env python3
"""Wait-count audit of gfx950 kernels from a `hipcc --save-temps` .s file.

  python scripts/waitcnt_audit.py <file.s> [kernel-substring ...] [--show]

Vector memory loads return in order, so an `s_waitcnt vmcnt(0)` waits for
every load in flight, prefetches included.  For every kernel: its loops
(a label and the backward branches to it), and per loop the static count of
vector loads, of `s_waitcnt` with vmcnt(0) / vmcnt(N > 0) / lgkmcnt(0), and
of barriers.  --show prints each vmcnt(0) with the instructions before it.
"""
import argparse
import re
import subprocess


def demangle(name):
    try:
        return subprocess.run(["c++filt"], input=name, capture_output=True, text=True).stdout.strip()
    except OSError:
        return name


def kernels(path):
    cur, body = None, []
    for line in open(path):
        m = re.match(r"^([A-Za-z_][\w.$]*):\s*(;.*)?$", line)
        if m and "_Z" in m.group(1) and not m.group(1).startswith("."):
            if cur:
                yield cur, body
            cur, body = m.group(1), []
            continue
        if cur is not None:
            if re.match(r"^\.Lfunc_end\d+:", line):
                yield cur, body
                cur, body = None, []
            else:
                body.append(line.rstrip("\n"))
    if cur:
        yield cur, body


LOAD = re.compile(r"^\s+(global_load|buffer_load|flat_load|global_atomic|scratch_load)")
STORE = re.compile(r"^\s+(global_store|buffer_store|flat_store|scratch_store)")


def audit(body, show):
    labels = {}
    for i, ln in enumerate(body):
        m = re.match(r"^(\.LBB\d+_\d+):", ln)
        if m:
            labels[m.group(1)] = i
    loops = []
    for i, ln in enumerate(body):
        m = re.match(r"^\s+s_(cbranch_\w+|branch)\s+(\.LBB\d+_\d+)", ln)
        if m and m.group(2) in labels and labels[m.group(2)] < i:
            loops.append((labels[m.group(2)], i))
    rows = []
    for a, b in sorted(set(loops)):
        seg = body[a:b + 1]
        w0 = [k for k, ln in enumerate(seg) if re.search(r"s_waitcnt.*vmcnt\(0\)", ln)]
        wn = sum(1 for ln in seg if re.search(r"s_waitcnt.*vmcnt\([1-9]\d*\)", ln))
        lg = sum(1 for ln in seg if re.search(r"s_waitcnt.*lgkmcnt\(0\)", ln))
        rows.append(dict(first=a, last=b, lines=b - a, loads=sum(1 for ln in seg if LOAD.match(ln)),
                         stores=sum(1 for ln in seg if STORE.match(ln)), vmcnt0=len(w0), vmcntN=wn, lgkm0=lg,
                         barriers=sum(1 for ln in seg if "s_barrier" in ln), w0_at=[a + k for k in w0]))
    return rows


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("s")
    ap.add_argument("match", nargs="*")
    ap.add_argument("--show", action="store_true")
    args = ap.parse_args()
    for name, body in kernels(args.s):
        dn = demangle(name)
        if args.match and not any(m in dn for m in args.match):
            continue
        tot0 = sum(1 for ln in body if re.search(r"s_waitcnt.*vmcnt\(0\)", ln))
        print(f"== {dn.split('(')[0]}: {len(body)} lines, {sum(1 for ln in body if LOAD.match(ln))} loads, "
              f"{tot0} vmcnt(0) in all")
        for r in audit(body, args.show):
            print(f"   loop [{r['first']}, {r['last']}] {r['lines']} lines: loads {r['loads']} stores {r['stores']} "
                  f"vmcnt(0) {r['vmcnt0']} vmcnt(N) {r['vmcntN']} lgkmcnt(0) {r['lgkm0']} barriers {r['barriers']}")
            if args.show:
                for k in r["w0_at"]:
                    ctx = [ln.strip() for ln in body[max(0, k - 4):k + 1]]
                    print("      @%d: %s" % (k, " | ".join(ctx)))


if __name__ == "__main__":
    main()
