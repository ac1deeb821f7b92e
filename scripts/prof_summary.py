"""Turn a scripts/gpu_prof.sh run into committed profile summaries.

    python scripts/prof_summary.py gpurun_out/<run> profiles/<tag>

writes
  <tag>_kernel_stats.csv      rocprofv3 --kernel-trace --stats of the short bench run, as produced
  <tag>_ntt_kernel_stats.csv  the same for the config 2 NTT leg (scripts/prof_ntt.py)
  <tag>_pmc.json              per kernel of the bench run: launches, mean duration, HBM bytes per
                              launch, L2 hit rate, SQ wait / VALU fractions
  <tag>_ntt_pmc.json          the same for the NTT leg
  <tag>_gemv_kernel_stats.csv, <tag>_gemv_pmc.json  the same for the gemv leg (scripts/gemv_time.py)
  <tag>_bench.json            the default bench line of the same run (when present)

Units and corrections (MI355X_MICROARCH.md, HBM section): FETCH_SIZE and
WRITE_SIZE are KiB; on gfx950 FETCH_SIZE reports half the bytes of a wide
coalesced streaming read, so fetch bytes = 2 x 1024 x FETCH_SIZE (validated
per access width by scripts/ubench_mem.hip, profiles/r2_fetch_calibration.txt).
VALU busy uses the gfx94x VALUBusy formula (ROCm 7.2 ships no gfx950 derived
counters): SQ_ACTIVE_INST_VALU x 4 / SIMDs / (GRBM_GUI_ACTIVE / 8 XCDs), with
1024 SIMDs (256 CUs x 4); GRBM_GUI_ACTIVE is summed over the 8 XCDs.
"""
import collections
import csv
import json
import os
import shutil
import sys

SIMDS = 1024
XCDS = 8


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


def summarise(run, prefix):
    dur = collections.defaultdict(list)
    for r in csv.DictReader(open(os.path.join(run, prefix + "kt", prefix + "kt_kernel_trace.csv"))):
        dur[short(r["Kernel_Name"])].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    pmc = {}
    for f in ("fetch", "write", "hit", "sq", "f64"):
        d = prefix + f
        for k, cs in counters(os.path.join(run, d, d + "_counter_collection.csv")).items():
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
            e["hbm_GBs"] = e["hbm_bytes"] / e["mean_us"] / 1e3
        if c.get("TCC_HIT_sum", 0) + c.get("TCC_MISS_sum", 0) > 0:
            e["l2_hit_rate"] = c["TCC_HIT_sum"] / (c["TCC_HIT_sum"] + c["TCC_MISS_sum"])
        if c.get("SQ_WAVE_CYCLES"):
            for q in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU"):
                if q in c:
                    e[q.lower() + "_frac"] = c[q] / c["SQ_WAVE_CYCLES"]
            e["sq_wait_any"] = e.get("sq_wait_any_frac")
        if c.get("GRBM_GUI_ACTIVE") and "SQ_ACTIVE_INST_VALU" in c:
            e["valu_busy"] = c["SQ_ACTIVE_INST_VALU"] * 4 / SIMDS / (c["GRBM_GUI_ACTIVE"] / XCDS)
            e["clock_GHz"] = c["GRBM_GUI_ACTIVE"] / XCDS / (e["mean_us"] * 1e3)
            # VALU issue fraction from the instruction count: every FP64 VALU
            # instruction of a wave64 holds the SIMD-32's FP64 pipe 4 cycles
            # (78.6 TF = 256 CUs x 4 SIMDs x 16 FMA lanes x 2 x 2.4 GHz)
            e["valu_frac"] = c["SQ_INSTS_VALU"] * 4 / SIMDS / (c["GRBM_GUI_ACTIVE"] / XCDS)
        f64 = [c.get("SQ_INSTS_VALU_" + x) for x in ("FMA_F64", "MUL_F64", "ADD_F64", "TRANS_F64")]
        if all(v is not None for v in f64):
            e["valu_mix"] = {k.lower(): c["SQ_INSTS_VALU_" + k] for k in
                             ("FMA_F64", "MUL_F64", "ADD_F64", "TRANS_F64", "INT32", "INT64", "CVT") if "SQ_INSTS_VALU_" + k in c}
        for q in ("SQ_INSTS_VALU", "SQ_INSTS_LDS", "SQ_BUSY_CYCLES"):
            if q in c:
                e[q.lower()] = c[q]
        out[k] = e
    return dict(sorted(out.items(), key=lambda kv: -kv[1]["mean_us"] * kv[1]["launches"]))


def main(run, tag):
    os.makedirs(os.path.dirname(tag) or ".", exist_ok=True)
    meta = {"source": run, "fetch_correction": "x2 (gfx950 FETCH_SIZE halves wide reads)",
            "units": "bytes per launch", "valu_busy": "SQ_ACTIVE_INST_VALU*4/1024/(GRBM_GUI_ACTIVE/8)",
            "valu_frac": "SQ_INSTS_VALU*4/1024/(GRBM_GUI_ACTIVE/8) (4 cycles per wave64 FP64 instruction)",
            "mean_us": "kernel trace of a bench run with the bench's own --steps 10 --warmup 2"}
    full = os.path.join(run, "bench_full.log")
    if os.path.exists(full):
        lines = [l for l in open(full) if l.startswith('{"metric"')]
        if lines:
            b = json.loads(lines[-1])
            json.dump(b, open(tag + "_bench.json", "w"), indent=1)
            meta["bench_workload"] = b["config"]["workload"]
            meta["pairs_per_launch"] = b["config"].get("pairs_per_launch")
    for prefix, suffix in (("", ""), ("ntt_", "_ntt"), ("gemv_", "_gemv")):
        if not os.path.exists(os.path.join(run, prefix + "kt")):
            continue
        shutil.copy(os.path.join(run, prefix + "kt", prefix + "kt_kernel_stats.csv"), tag + suffix + "_kernel_stats.csv")
        out = summarise(run, prefix)
        m = dict(meta)
        if prefix:
            m = {k: v for k, v in meta.items() if k not in ("bench_workload", "pairs_per_launch")}
            m["workload"] = ("config 2: NTT -> INTT of 1024 polys, N=2^16, L=8 (scripts/prof_ntt.py)" if prefix == "ntt_"
                             else "he_gemv_batch of 256 ciphertexts, N=2^16, L=8, 16 slots, bench51 primes "
                                  "(scripts/gemv_time.py --count 256 --rot 0; the bench's gemv leg)")
            if prefix == "gemv_":
                m["cts_per_launch"] = 256
                m["mean_us"] = "kernel trace of the same command"
        json.dump({"meta": m, "kernels": out}, open(tag + suffix + "_pmc.json", "w"), indent=1)
        print(f"== {tag}{suffix}")
        for k, e in list(out.items())[:14]:
            print(f"{k:40s} n={e['launches']:4d} {e['mean_us']:8.1f} us  hbm={e.get('hbm_bytes', 0) / 1e6:8.1f} MB "
                  f"({e.get('hbm_GBs', 0):6.0f} GB/s) l2hit={e.get('l2_hit_rate', 0):.2f} "
                  f"wait={e.get('sq_wait_any_frac', 0) or 0:.2f} valu={e.get('valu_busy', 0):.2f}")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
