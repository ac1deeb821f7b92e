"""Time he_gemv / he_gemv_batch / he_rot_batch at a large ring (MI355X).

python scripts/gemv_time.py [--set bench51] [--slots 16] [--count 8] [--reps 3]
Prints one JSON line: per-gemv and per-rotation microseconds of the single
call (he_gemv) and of the batch entry points on `count` random-residue
ciphertexts (uniform residues: the cost does not depend on the values).
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--set", default="bench51")
    ap.add_argument("--slots", type=int, default=16)
    ap.add_argument("--count", type=int, default=8)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--single", type=int, default=1)
    ap.add_argument("--rot", type=int, default=1, help="0: he_gemv_batch only (profiling passes of the gemv leg)")
    args = ap.parse_args()
    import numpy as np
    import torch
    from hectr_amd.gpqhe import Engine
    from tests.test_gpu_parity import PARAMS
    e = Engine.product()
    kw = dict(PARAMS[args.set][1], slots=args.slots)
    e.init_params(**kw)
    e.set_seed(5)
    pk, sk = e.pk(), e.sk()
    e.keypair(pk, sk)
    rk = e.evks(e.slots)
    e.genrk(rk, sk)
    n, L, s, cnt = e.n, e.L, e.slots, args.count
    rng = np.random.default_rng(1)
    M = np.ascontiguousarray((rng.uniform(-1, 1, (s, s)) + 0j).ravel())
    x = torch.empty(cnt * 2 * L * n, dtype=torch.int64, device="cuda")
    torch.cuda.synchronize()
    e.lib.poly_fill_uniform(x.data_ptr(), 2 * cnt, L, 3)
    y = torch.empty(cnt * 2 * (L - 1) * n, dtype=torch.int64, device="cuda")
    r = torch.empty(cnt * 2 * L * n, dtype=torch.int64, device="cuda")
    out = {"set": args.set, "n": n, "L": L, "slots": s, "count": cnt}

    def timed(fn):
        fn()
        e.sync()
        best = 1e30
        for _ in range(args.reps):
            t0 = time.perf_counter()
            fn()
            e.sync()
            best = min(best, time.perf_counter() - t0)
        return best

    t = timed(lambda: e.lib.he_gemv_batch(y.data_ptr(), M.ctypes.data, x.data_ptr(), cnt, L, rk))
    out["gemv_batch_us_per_ct"] = t / cnt * 1e6
    if args.rot:
        t = timed(lambda: e.lib.he_rot_batch(r.data_ptr(), x.data_ptr(), cnt, L, 1, rk))
        out["rot_batch_us_per_ct"] = t / cnt * 1e6
    # per-kernel device time of one batch of each (HIP events on the engine stream)
    for name, fn in (("gemv_batch", lambda: e.lib.he_gemv_batch(y.data_ptr(), M.ctypes.data, x.data_ptr(), cnt, L,
                                                                 rk)),
                     ("rot_batch", lambda: e.lib.he_rot_batch(r.data_ptr(), x.data_ptr(), cnt, L, 1, rk))):
        if name == "rot_batch" and not args.rot:
            continue
        e.prof_enable(True)
        fn()
        e.sync()
        st = e.prof_collect()
        e.prof_enable(False)
        out[name + "_kernels_us_per_ct"] = {k: round(v[1] / cnt, 2) for k, v in sorted(st.items(),
                                                                                      key=lambda kv: -kv[1][1])}
        out[name + "_kernels_GBs"] = {k: round(v[2] / v[1] / 1e3, 1) for k, v in st.items() if v[1] > 0}
    if args.single:
        ct = e.encrypt(rng.uniform(-1, 1, s) + 0j, pk)
        yc = e.ct()
        out["gemv_single_us"] = timed(lambda: e.gemv(yc, M, ct, rk)) * 1e6
        out["rot_single_us"] = timed(lambda: e.rot(yc, ct, 1, rk)) * 1e6
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
