"""Host time per Engine method inside the encrypted CSTR regulator (config 4):
where the wall time of a step goes when the GPU timeline is shorter."""
import collections
import sys
import time

sys.path.insert(0, ".")
import numpy as np

from hectr_amd.cstr import CstrProblem, EncryptedRegulator
from hectr_amd.gpqhe import Engine

steps = int(sys.argv[1]) if len(sys.argv) > 1 else 100
pb = CstrProblem(steps)
eng = Engine.product()
reg = EncryptedRegulator(eng, pb, seed=5)
pb.simulate(reg)
acc = collections.defaultdict(lambda: [0, 0.0])
for name in ("ecd", "enc_pk", "free", "ct", "pt", "sub", "gemv", "add", "neg", "copy_ct", "moddown", "dec", "dcd"):
    f = getattr(eng, name)

    def wrap(*a, _f=f, _n=name, **k):
        t0 = time.perf_counter()
        r = _f(*a, **k)
        acc[_n][0] += 1
        acc[_n][1] += time.perf_counter() - t0
        return r
    setattr(eng, name, wrap)
reg.timings.clear()
t0 = time.perf_counter()
pb.simulate(reg)
dt = time.perf_counter() - t0
tot = sum(v[1] for v in acc.values())
print(f"steps {steps}: wall {dt * 1e3 / steps:.3f} ms/step, regulator median {1e3 * np.median(reg.timings):.3f} ms, "
      f"engine calls {tot * 1e3 / steps:.3f} ms/step")
for k, v in sorted(acc.items(), key=lambda kv: -kv[1][1]):
    print(f"  {k:10s} {v[0] / steps:5.1f} calls/step {v[1] * 1e6 / steps:8.1f} us/step")
reg.close()
eng.exit()
