"""Debug: GPU encoder (GPQHE_GPU_ECD_MIN=2) vs oracle for growing slot counts."""
import os
import sys

os.environ["GPQHE_GPU_ECD_MIN"] = "2"
sys.path.insert(0, ".")
import numpy as np

from hectr_amd.gpqhe import Engine
from tests.test_gpu_parity import PARAMS

o, p = Engine.oracle(), Engine.product()
for e in (o, p):
    e.init_params(**PARAMS["c1"][1])
    e.set_seed(1)
n, L = o.n, o.L
for s in (2, 4, 8, 16, 64, 256, 1024, 2048, 4096):
    z = np.arange(s) * 0.001 + 0.5 + 0.25j
    out = {}
    for e in (o, p):
        pt = e.pt()
        e.ecd_ex(pt, z, s, o.info.delta, L)
        r = e.export(pt).reshape(L, n).copy()
        o.lib.poly_intt_batch(r.ctypes.data, 1, L)
        q0 = o.primes[0]
        out[e.name] = np.array([int(x) - q0 if int(x) > q0 // 2 else int(x) for x in r[0]])
        e.free(pt)
    bad = np.flatnonzero(out["oracle"] != out["product"])
    print(s, "mismatch", bad.size, "first", bad[:4], out["oracle"][bad[:2]] if bad.size else "",
          out["product"][bad[:2]] if bad.size else "", flush=True)
