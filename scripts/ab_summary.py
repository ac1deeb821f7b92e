"""Summarise bench logs (a gpurun_out/<run> directory or log files): value,
60-bit / config-5 values and the per-kernel table."""
import glob
import json
import os
import sys

files = []
for a in sys.argv[1:]:
    files += sorted(glob.glob(os.path.join(a, "bench_*.log"))) if os.path.isdir(a) else [a]
for f in files:
    line = [l for l in open(f) if l.startswith('{"metric"')]
    if not line:
        print(f, "NO RESULT")
        continue
    d = json.loads(line[-1])
    ks = sorted(d.get("kernels", {}).items(), key=lambda kv: -kv[1]["share"])
    extra = ""
    if "value_60bit" in d:
        extra += f"  60-bit {d['value_60bit']:.0f}"
    if "config5" in d:
        extra += f"  c5 {d['config5']['value']:.0f}"
        if "value_60bit" in d["config5"]:
            extra += f"  c5-60bit {d['config5']['value_60bit']:.0f}"
    g = d.get("gemv")
    if g:
        extra += f"  gemv {g['value']:.0f}"
        if "alt_primes" in g:
            extra += f" (60-bit {g['alt_primes']['value']:.0f})"
    h = d.get("config5", {}).get("hempc_gemv")
    if h:
        extra += f"  c5-gemv {h['value']:.0f}"
    c = d.get("cstr")
    if c:
        extra += f"  cstr-py {c['steps_per_s']:.0f}/s (spec {c.get('spec_gemv_taken')})"
        cc = c.get("c_caller") or {}
        if "closed_loop_ms_median" in cc:
            extra += f"  C-harness {cc['closed_loop_ms_median']:.3f} ms/40"
            c4 = cc.get("config4_c_driver") or {}
            if "steps_per_s" in c4:
                extra += f"  c4-driver {c4['steps_per_s']:.0f}/s"
    print(f"{os.path.basename(f):16s} {d['value']:9.0f} {d['unit']}{extra}  ms/step {d['ms_per_step']:.3f}")
    if "ntt_roundtrip" in d:
        t = d["ntt_roundtrip"]
        print(f"    ntt roundtrip {t['polys']} polys: {t['roundtrip_ms']:.2f} ms, {t['alg_GBs']:.0f} GB/s")
    for k, v in ks:
        print(f"    {k:28s} {v['launches']:5d} x {v['avg_us']:8.1f} us  {v['share']*100:5.1f}%  {v['streamed_GBs']:7.0f} GB/s")
