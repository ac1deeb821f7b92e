"""Turn a scripts/gpu_prof.sh run into committed profile summaries.

    python scripts/prof_summary.py gpurun_out/<run> profiles/<tag>

writes <tag>_kernel_stats.csv (rocprofv3 --kernel-trace --stats, as produced),
<tag>_pmc.json (per kernel: launches, mean duration, HBM bytes per launch from
FETCH_SIZE / WRITE_SIZE, L2 hit rate, SQ wait fractions) and, when the run
has one, <tag>_bench.json (the default bench line of the same run).

Units and corrections (MI355X_MICROARCH.md, HBM section): FETCH_SIZE and
WRITE_SIZE are KiB; on gfx950 FETCH_SIZE reports half the bytes of a wide
coalesced streaming read, so fetch bytes = 2 x 1024 x FETCH_SIZE.
"""
import collections
import csv
import json
import os
import shutil
import sys


def short(name):
    name = name.split("(")[0]
    return name[5:] if name.startswith("void ") else name


def counters(path):
    per = collections.defaultdict(lambda: collections.defaultdict(list))
    if not os.path.exists(path):
        return per
    for r in csv.DictReader(open(path)):
        per[short(r["Kernel_Name"])][r["Counter_Name"]].append(float(r["Counter_Value"]))
    return per


def main(run, tag):
    os.makedirs(os.path.dirname(tag) or ".", exist_ok=True)
    shutil.copy(os.path.join(run, "kt", "kt_kernel_stats.csv"), tag + "_kernel_stats.csv")
    dur = collections.defaultdict(list)
    for r in csv.DictReader(open(os.path.join(run, "kt", "kt_kernel_trace.csv"))):
        dur[short(r["Kernel_Name"])].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    pmc = {}
    for f in ("fetch", "write", "hit", "sq"):
        for k, cs in counters(os.path.join(run, f, f + "_counter_collection.csv")).items():
            for c, v in cs.items():
                pmc.setdefault(k, {})[c] = sum(v) / len(v)
    out = {}
    for k, d in dur.items():
        e = {"launches": len(d), "mean_us": sum(d) / len(d)}
        c = pmc.get(k, {})
        if "FETCH_SIZE" in c:
            e["hbm_read_bytes"] = 2 * 1024 * c["FETCH_SIZE"]
        if "WRITE_SIZE" in c:
            e["hbm_write_bytes"] = 1024 * c["WRITE_SIZE"]
        if "hbm_read_bytes" in e and "hbm_write_bytes" in e:
            e["hbm_bytes"] = e["hbm_read_bytes"] + e["hbm_write_bytes"]
        if c.get("TCC_HIT_sum", 0) + c.get("TCC_MISS_sum", 0) > 0:
            e["l2_hit_rate"] = c["TCC_HIT_sum"] / (c["TCC_HIT_sum"] + c["TCC_MISS_sum"])
        if c.get("SQ_WAVE_CYCLES"):
            for q in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY"):
                e[q.lower() + "_frac"] = c[q] / c["SQ_WAVE_CYCLES"]
        out[k] = e
    meta = {"source": run, "fetch_correction": "x2 (gfx950 FETCH_SIZE halves wide reads)", "units": "bytes per launch"}
    bench_cfg = None
    full = os.path.join(run, "bench_full.log")
    if os.path.exists(full):
        lines = [l for l in open(full) if l.startswith('{"metric"')]
        if lines:
            b = json.loads(lines[-1])
            json.dump(b, open(tag + "_bench.json", "w"), indent=1)
            bench_cfg = b["config"]["workload"]
    meta["bench_workload"] = bench_cfg
    json.dump({"meta": meta, "kernels": dict(sorted(out.items(), key=lambda kv: -kv[1]["mean_us"] * kv[1]["launches"]))},
              open(tag + "_pmc.json", "w"), indent=1)
    for k, e in sorted(out.items(), key=lambda kv: -kv[1]["mean_us"] * kv[1]["launches"])[:14]:
        print(f"{k:40s} n={e['launches']:4d} {e['mean_us']:8.1f} us  "
              f"hbm={e.get('hbm_bytes', 0) / 1e6:8.1f} MB  l2hit={e.get('l2_hit_rate', 0):.2f} "
              f"wait={e.get('sq_wait_any_frac', 0):.2f}")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
