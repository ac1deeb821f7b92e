#!/usr/bin/env python3
"""Static instruction mix of gfx950 kernels from a `hipcc --save-temps` .s file.

  python scripts/isa_count.py <file.s> <kernel-name-substring> [--top N]

Per kernel: instruction counts by class (FP64 VALU, other VALU, SALU, LDS,
vector memory, branches) and the most frequent mnemonics, plus the
compiler's register / spill metadata.  Static counts: a loop body is counted
once, so compare kernels of the same structure, or use SQ_INSTS_* PMC for the
dynamic totals.
"""
import argparse
import collections
import re
import subprocess


def demangle(names):
    try:
        out = subprocess.run(["c++filt"], input="\n".join(names), capture_output=True, text=True).stdout
        return out.splitlines()
    except OSError:
        return names


def kernels(path):
    cur, body = None, []
    for line in open(path):
        m = re.match(r"^([A-Za-z_][\w.$]*):\s*(;.*)?$", line)
        if m and not m.group(1).startswith(".") and "_Z" in m.group(1):
            if cur:
                yield cur, body
            cur, body = m.group(1), []
            continue
        if cur is not None:
            if line.startswith("\t.end_amdgpu_metadata") or re.match(r"^\.Lfunc_end\d+:", line):
                yield cur, body
                cur, body = None, []
            else:
                body.append(line)
    if cur:
        yield cur, body


def classify(mn):
    if mn.startswith("v_"):
        if "_f64" in mn or mn in ("v_rndne_f64", "v_trunc_f64", "v_floor_f64"):
            return "valu_f64"
        if mn.startswith("v_mfma"):
            return "mfma"
        return "valu_other"
    if mn.startswith("s_waitcnt") or mn.startswith("s_barrier") or mn.startswith("s_nop"):
        return "wait/sync"
    if mn.startswith("s_cbranch") or mn.startswith("s_branch"):
        return "branch"
    if mn.startswith("s_"):
        return "salu/smem"
    if mn.startswith("ds_"):
        return "lds"
    if mn.startswith(("global_", "buffer_", "flat_", "scratch_")):
        return "vmem"
    return "other"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("asm")
    ap.add_argument("pattern")
    ap.add_argument("--top", type=int, default=25)
    a = ap.parse_args()
    ks = list(kernels(a.asm))
    dem = demangle([k for k, _ in ks])
    for (name, body), dn in zip(ks, dem):
        if a.pattern not in dn:
            continue
        cls, mns = collections.Counter(), collections.Counter()
        meta = {}
        for line in body:
            s = line.strip()
            if not s or s.startswith((";", ".")) or s.endswith(":"):
                m = re.match(r";\s*(NumVgprs|NumAgprs|ScratchSize|Occupancy|NumSgprs|TotalNumVgprs):\s*(\d+)", s)
                if m:
                    meta[m.group(1)] = int(m.group(2))
                continue
            mn = s.split()[0]
            mns[mn] += 1
            cls[classify(mn)] += 1
        print(f"== {dn}")
        print("   meta:", meta)
        print("   classes:", dict(cls), "total", sum(cls.values()))
        for mn, c in mns.most_common(a.top):
            print(f"   {c:6d} {mn}")


if __name__ == "__main__":
    main()
