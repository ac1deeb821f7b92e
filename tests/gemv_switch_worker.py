"""Child process of the GPU tests whose library switches are read once per
process (test infrastructure only).  Prints one JSON line.

  gemv_switch_worker.py [generic]   he_gemv_batch / he_rot_batch at N=2^16,
      L=8 (bench51, 16 slots) under the environment it was started with
      (GPQHE_GEMV_WIN=0: the per-ciphertext generic kernels instead of the
      windowed batch path): {case: number of residues differing from the
      oracle}
  gemv_switch_worker.py foldcap     (GPQHE_FOLD_MIB small) a dense 256-slot
      matrix at n = 2^13 whose folded key set exceeds the cap, through
      he_gemv_batch and he_gemv, and a 16-diagonal one that still folds:
      {case: differing residues}
  gemv_switch_worker.py teardown    the two-stream he_mul_rescale_batch, then
      hectx_exit (which releases the second stream, its events and the
      context's stream), a second context in the same process on one stream,
      hectx_exit again: {"equal": outputs of the two contexts equal}
"""
import ctypes
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from hectr_amd.gpqhe import Engine  # noqa: E402
from tests.test_gpu_rotations import (encrypt_batch, init_slots, rot_keys, run_batch,  # noqa: E402
                                      sample_matrix)


def generic(ora, prod):
    init_slots(ora, prod, "bench51", 16, seed=53)
    s, n, lvl, cnt = 16, prod.n, 8, 2
    ko, kp = rot_keys(ora), rot_keys(prod)
    rng = np.random.default_rng(9)
    zs = rng.uniform(-1, 1, (cnt, s)) + 1j * rng.uniform(-1, 1, (cnt, s))
    Mc = np.ascontiguousarray(sample_matrix(s, 4).ravel(), dtype=np.complex128)
    host = encrypt_batch(prod, kp[0], zs, nlimbs=lvl)
    out = {}
    want, got = run_batch(ora, prod, ko[2], kp[2], "he_gemv_batch", host, cnt * 2 * (lvl - 1) * n,
                          Mc.ctypes.data, "IN", cnt, lvl)
    out["gemv_batch"] = int(np.count_nonzero(got != want))
    want, got = run_batch(ora, prod, ko[2], kp[2], "he_rot_batch", host, cnt * 2 * lvl * n, "IN", cnt, lvl, 5)
    out["rot_batch"] = int(np.count_nonzero(got != want))
    return out


def foldcap(ora, prod):
    s = 256
    init_slots(ora, prod, "f13", s, seed=61)
    n, lvl, cnt = prod.n, 6, 2
    ko, kp = rot_keys(ora), rot_keys(prod)
    rng = np.random.default_rng(13)
    zs = rng.uniform(-1, 1, (cnt, s)) + 1j * rng.uniform(-1, 1, (cnt, s))
    dense = rng.uniform(-1, 1, (s, s)) + 1j * rng.uniform(-1, 1, (s, s))
    sparse = dense * np.isin(np.add.outer(-np.arange(s), np.arange(s)) % s, np.arange(0, s, 16))
    host = encrypt_batch(prod, kp[0], zs, nlimbs=lvl)
    out = {}
    for name, M in (("gemv_batch_dense", dense), ("gemv_batch_sparse", sparse)):
        Mc = np.ascontiguousarray(M.ravel(), dtype=np.complex128)
        want, got = run_batch(ora, prod, ko[2], kp[2], "he_gemv_batch", host, cnt * 2 * (lvl - 1) * n,
                              Mc.ctypes.data, "IN", cnt, lvl)
        out[name] = int(np.count_nonzero(got != want))
    res = {}
    for e, (pk, sk, rk) in ((ora, ko), (prod, kp)):
        x, y = e.ct(), e.ct()
        e.import_(x, host.reshape(cnt, -1)[0], lvl, scale=prod.info.delta)
        e.gemv(y, dense.ravel(), x, rk)
        res[e.name] = e.export(y)
    out["gemv_dense"] = int(np.count_nonzero(res["oracle"] != res["product"]))
    return out


def teardown(ora, prod):
    from tests.test_gpu_parity import PARAMS
    import torch
    kw = PARAMS["bench51"][1]
    cnt, outs = 8, []
    for streams in (2, 1):
        prod.init_params(**kw)
        prod.set_seed(5)
        pk, sk = prod.pk(), prod.sk()
        prod.keypair(pk, sk)
        rlk = prod.evk()
        prod.genrlk(rlk, sk)
        n, lvl = prod.n, prod.L
        a = torch.empty(cnt * 2 * lvl * n, dtype=torch.int64, device="cuda")
        b = torch.empty_like(a)
        o = torch.full((cnt * 2 * (lvl - 1) * n,), 7, dtype=torch.int64, device="cuda")
        torch.cuda.synchronize()
        prod.lib.poly_fill_uniform(a.data_ptr(), 2 * cnt, lvl, 1)
        prod.lib.poly_fill_uniform(b.data_ptr(), 2 * cnt, lvl, 2)
        prod.lib.gpqhe_set_streams(streams)
        prod.lib.he_mul_rescale_batch(o.data_ptr(), a.data_ptr(), b.data_ptr(), cnt, lvl, ctypes.byref(rlk))
        prod.sync()
        outs.append(o.cpu().numpy())
        prod.exit()  # objects outliving the context: their blocks went with its pool
        del a, b, o
    return {"equal": bool(np.array_equal(outs[0], outs[1]))}


def main():
    import torch
    assert torch.cuda.is_available()  # torch's HIP initialisation before the library's (as conftest's fixture)
    torch.cuda.init()
    ora, prod = Engine.oracle(), Engine.product()
    case = sys.argv[1] if len(sys.argv) > 1 else "generic"
    print(json.dumps({"generic": generic, "foldcap": foldcap, "teardown": teardown}[case](ora, prod)), flush=True)


if __name__ == "__main__":
    main()
