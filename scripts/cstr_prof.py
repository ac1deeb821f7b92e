"""Device time vs wall time of the encrypted CSTR loop (config 4) per step."""
import sys
import time

sys.path.insert(0, ".")
import numpy as np

from hectr_amd.cstr import CstrProblem, EncryptedRegulator
from hectr_amd.gpqhe import Engine

steps = int(sys.argv[1]) if len(sys.argv) > 1 else 100
prof = not (len(sys.argv) > 2 and sys.argv[2] == "noprof")  # noprof: for rocprofv3 --kernel-trace
pb = CstrProblem(steps)
eng = Engine.product()
reg = EncryptedRegulator(eng, pb, seed=5)
pb.simulate(reg)  # warm: diagonal cache, pool, code objects
reg.timings.clear()
eng.prof_enable(prof)
t0 = time.perf_counter()
x, u = pb.simulate(reg)
dt = time.perf_counter() - t0
stats = eng.prof_collect()
eng.prof_enable(False)
dev = sum(v[1] for v in stats.values())
launches = sum(v[0] for v in stats.values())
print(f"steps {steps}: wall {dt * 1e3 / steps:.3f} ms/step, regulator median {1e3 * np.median(reg.timings):.3f} ms, "
      f"device {dev / 1e3 / steps:.3f} ms/step, launches/step {launches / steps:.1f}")
for k, v in sorted(stats.items(), key=lambda kv: -kv[1][1]):
    print(f"  {k:28s} {v[0] / steps:6.1f} launches/step  {v[1] / steps:8.1f} us/step")
reg.close()
eng.exit()
