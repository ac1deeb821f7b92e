"""Summarise gpurun_out/<run>/bench_*.log files: value and top kernels."""
import glob
import json
import sys

for f in sorted(glob.glob(f"gpurun_out/{sys.argv[1]}/bench_*.log")):
    line = [l for l in open(f) if l.startswith('{"metric"')]
    if not line:
        print(f, "NO RESULT")
        continue
    d = json.loads(line[0])
    ks = sorted(d.get("kernels", {}).items(), key=lambda kv: -kv[1]["share"])
    print(f"{f.split('/')[-1]:24s} {d['value']:9.0f} {d['unit']}  dom={d['roofline']['kernel']} "
          f"{d['roofline']['achieved']:.0f} GB/s")
    if "ntt_roundtrip" in d:
        t = d["ntt_roundtrip"]
        print(f"    ntt roundtrip {t['polys']} polys: {t['roundtrip_ms']:.2f} ms, {t['alg_GBs']:.0f} GB/s")
    for k, v in ks:
        print(f"    {k:28s} {v['avg_us']:8.1f} us  {v['share']*100:5.1f}%  {v['streamed_GBs']:7.0f} GB/s")
