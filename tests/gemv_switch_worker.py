"""Child process of test_gemv_generic_path: he_gemv, he_rot and their batch
entry points at N=2^16, L=8 (bench51, 16 slots) on the oracle and on the
product library under the environment it was started with (GPQHE_GEMV_WIN=0:
the per-ciphertext generic kernels instead of the windowed batch path), and
prints one JSON line {case: number of differing residues}.  Test
infrastructure only."""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from hectr_amd.gpqhe import Engine  # noqa: E402
from tests.test_gpu_rotations import (encrypt_batch, init_slots, rot_keys, run_batch,  # noqa: E402
                                      sample_matrix)


def main():
    import torch
    assert torch.cuda.is_available()  # torch's HIP initialisation before the library's (as conftest's fixture)
    torch.cuda.init()
    ora, prod = Engine.oracle(), Engine.product()
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
    print(json.dumps(out))


if __name__ == "__main__":
    main()
