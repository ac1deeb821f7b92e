"""he_gemv_batch / he_rot_batch at the shapes bench.py times, the Galois
orbit wrap, in-place calls and the fold-size fallback: product (libgpqhe.so
on MI355X) vs oracle, bit for bit, decoded against M @ z and np.roll.

HECTR's hot call is he_gemv (reference src/hempc.c:257-259) with `slots`
rotation keys (src/ctr.c:521,526-532).  test_gpu_rotations.py pins the path
at 3-17 ciphertexts; here:

* the bench's own batch sizes: 256 ciphertexts at N=2^16, L=8 on bench51 and
  bench_d2 (bench.py --gemv-batch, and its he_rot_batch by 1) and 64 at
  N=2^17, L=12 on c5f (--c5-gemv-batch, config5.hempc_gemv).  The inner
  product kernel's grid depends on the count: ceil(count / C) member groups
  per XCD group, the last group's partial member count;
* n = 2^13 (64 blocks per orbit) with 256 and 512 slots: rotations of 64 and
  more wrap the orbit (output block o reads source block o + d mod 64), and a
  dense 128- / 256-slot matrix runs as many launches of <= 16 diagonals;
* he_rot(c, c) and he_gemv(c, M, c) in place;
* a matrix whose folded key set exceeds GPQHE_FOLD_MIB takes the
  per-ciphertext path (child process: the cap is read once per process).
"""
import json
import os
import subprocess
import sys

import numpy as np
import pytest

from tests.test_gpu_parity import same
from tests.test_gpu_rotations import init_slots, rot_keys, run_batch, sample_matrix

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def encrypt_host(e, pk, zs, lvl):
    """Fresh encryptions of the rows of zs at level lvl, exported to one host
    array [count][2][lvl][n] (objects freed)."""
    out = np.empty((len(zs), 2 * lvl * e.n), dtype=np.uint64)
    for i, z in enumerate(zs):
        ct = e.encrypt(z, pk, nlimbs=lvl)
        out[i] = e.export(ct).ravel()
        e.free(ct)
    return out.ravel()


def decoded(product, words, lvl, sk):
    ct = product.ct()
    product.import_(ct, words, lvl, scale=product.info.delta)
    z = product.decrypt(ct, sk)
    product.free(ct)
    return z


@pytest.mark.parametrize("name,cnt,lvl", [("bench51", 256, 8), ("bench_d2", 256, 8), ("c5f", 64, 12)])
def test_gemv_rot_batch_bench_shape(oracle, product, name, cnt, lvl):
    """bench.py's gemv legs at their timed shapes: a dense 16-slot matrix
    (every diagonal non-zero, as GemvWork builds it) over `cnt` ciphertexts
    in one call, and he_rot_batch by 1 and by slots - 1 over the same batch;
    every output residue against the oracle, a spread of outputs decoded."""
    s = 16
    init_slots(oracle, product, name, s, seed=cnt + lvl)
    n = product.n
    ko, kp = rot_keys(oracle), rot_keys(product)
    rng = np.random.default_rng(cnt)
    zs = rng.uniform(-1, 1, (cnt, s)) + 1j * rng.uniform(-1, 1, (cnt, s))
    M = rng.uniform(-1, 1, (s, s)) + 1j * rng.uniform(-1, 1, (s, s))
    Mc = np.ascontiguousarray(M.ravel(), dtype=np.complex128)
    host = encrypt_host(product, kp[0], zs, lvl)
    want, got = run_batch(oracle, product, ko[2], kp[2], "he_gemv_batch", host, cnt * 2 * (lvl - 1) * n,
                          Mc.ctypes.data, "IN", cnt, lvl)
    assert np.array_equal(got, want), f"gemv: {np.count_nonzero(got != want)} residues differ"
    sk = kp[1]
    per = got.reshape(cnt, -1)
    for i in sorted({0, 1, cnt // 2, cnt - 2, cnt - 1}):
        ref = M @ zs[i]
        assert np.abs(decoded(product, per[i], lvl - 1, sk) - ref).max() < 1e-6 * max(1.0, np.abs(ref).max()), i
    del want, got, per
    for r in (1, s - 1):
        want, got = run_batch(oracle, product, ko[2], kp[2], "he_rot_batch", host, cnt * 2 * lvl * n, "IN", cnt, lvl, r)
        assert np.array_equal(got, want), f"rot {r}: {np.count_nonzero(got != want)} residues differ"
        per = got.reshape(cnt, -1)
        for i in (0, cnt - 1):
            assert np.abs(decoded(product, per[i], lvl, sk) - np.roll(zs[i], -r)).max() < 1e-6, (r, i)
        del want, got, per
    for e, k in ((oracle, ko), (product, kp)):
        e.free_evks(k[2])


@pytest.mark.parametrize("slots,rots,diags", [
    (256, (64, 100, 128, 255), "dense128"),
    (256, (63, 65, 192), "dense256"),
    (512, (64, 100, 256, 511), (0, 1, 63, 64, 65, 100, 257, 511)),
])
def test_orbit_wrap_n2_13(oracle, product, slots, rots, diags):
    """n = 2^13 on the all-FP64 set f13: P = 64 blocks per Galois orbit, so
    rotations of 64 and more (up to slots - 1) wrap the orbit, and a
    gemv with diagonals spread over [0, slots) runs launches of <= 16
    consecutive rotations.  he_rot_batch (3 ciphertexts) and he_gemv_batch
    against the oracle; decoded against np.roll and M @ z.  "dense128": a
    128 x 128 block of a 256-slot matrix (every diagonal non-zero),
    "dense256": the full 256 x 256 matrix."""
    init_slots(oracle, product, "f13", slots, seed=slots)
    s, n, lvl, cnt = slots, product.n, 6, 3
    ko, kp = rot_keys(oracle), rot_keys(product)
    for r in (1, 64, s - 1):
        same(oracle, product, ko[2][r], kp[2][r])
    rng = np.random.default_rng(s)
    zs = rng.uniform(-1, 1, (cnt, s)) + 1j * rng.uniform(-1, 1, (cnt, s))
    M = rng.uniform(-1, 1, (s, s)) + 1j * rng.uniform(-1, 1, (s, s))
    if diags == "dense128":
        M[128:, :] = 0
        M[:, 128:] = 0
    elif diags != "dense256":
        M *= np.isin(np.add.outer(-np.arange(s), np.arange(s)) % s, diags)
    Mc = np.ascontiguousarray(M.ravel(), dtype=np.complex128)
    host = encrypt_host(product, kp[0], zs, lvl)
    sk = kp[1]
    for r in rots:
        want, got = run_batch(oracle, product, ko[2], kp[2], "he_rot_batch", host, cnt * 2 * lvl * n, "IN", cnt, lvl, r)
        assert np.array_equal(got, want), f"rot {r}: {np.count_nonzero(got != want)} residues differ"
        z = decoded(product, got.reshape(cnt, -1)[cnt - 1], lvl, sk)
        assert np.abs(z - np.roll(zs[cnt - 1], -r)).max() < 1e-6, r
    want, got = run_batch(oracle, product, ko[2], kp[2], "he_gemv_batch", host, cnt * 2 * (lvl - 1) * n,
                          Mc.ctypes.data, "IN", cnt, lvl)
    assert np.array_equal(got, want), f"gemv: {np.count_nonzero(got != want)} residues differ"
    for i in range(cnt):
        ref = M @ zs[i]
        z = decoded(product, got.reshape(cnt, -1)[i], lvl - 1, sk)
        assert np.abs(z - ref).max() < 1e-6 * max(1.0, np.abs(ref).max()), i
    for e, k in ((oracle, ko), (product, kp)):
        e.free_evks(k[2])


@pytest.mark.parametrize("name,slots", [("bench51", 16), ("bench_d2", 16), ("f13", 256)])
def test_rot_gemv_in_place(oracle, product, name, slots):
    """he_rot(c, c, r) and he_gemv(c, M, c) with the output object the input
    (the windowed path reads every input word before its ModDown writes):
    residues equal the oracle's out-of-place results."""
    init_slots(oracle, product, name, slots, seed=19)
    s = slots
    ko, kp = rot_keys(oracle), rot_keys(product)
    rng = np.random.default_rng(7)
    z = rng.uniform(-1, 1, s) + 1j * rng.uniform(-1, 1, s)
    M = sample_matrix(s, 11)
    r = s - 1 if s <= 64 else 100
    res = {}
    for e, (pk, sk, rk) in ((oracle, ko), (product, kp)):
        x = e.encrypt(z, pk)
        if e is product:
            e.rot(x, x, r, rk)
            e.gemv(x, M.ravel(), x, rk)
            res[e.name] = e.export(x)
        else:
            a, b = e.ct(), e.ct()
            e.rot(a, x, r, rk)
            e.gemv(b, M.ravel(), a, rk)
            res[e.name] = e.export(b)
    assert np.array_equal(res["product"], res["oracle"]), \
        f"{np.count_nonzero(res['product'] != res['oracle'])} residues differ"
    x = product.ct()
    product.import_(x, res["product"], product.L - 1, scale=product.info.delta)
    got = product.decrypt(x, kp[1])
    ref = M @ np.roll(z, -r)
    assert np.abs(got - ref).max() < 1e-6 * max(1.0, np.abs(ref).max())
    for e, k in ((oracle, ko), (product, kp)):
        e.free_evks(k[2])


def run_worker(case, env_extra, timeout=600):
    env = dict(os.environ, **env_extra)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tests", "gemv_switch_worker.py"), case], env=env,
                       cwd=ROOT, capture_output=True, text=True, timeout=timeout)
    assert r.returncode == 0, f"rc {r.returncode}\n" + r.stdout[-2000:] + r.stderr[-3000:]
    return json.loads([x for x in r.stdout.splitlines() if x.startswith("{")][-1])


def test_gemv_fold_cap_fallback():
    """GPQHE_FOLD_MIB=256: a dense 256-slot matrix at n = 2^13 (f13: a folded
    set of ~700 MB) exceeds the cap, so he_gemv_batch and he_gemv run the
    per-ciphertext path (bounded diagonal cache) instead of aborting; a
    16-diagonal matrix still folds.  Bit-exact against the oracle."""
    res = run_worker("foldcap", {"GPQHE_FOLD_MIB": "256"})
    assert res == {"gemv_batch_dense": 0, "gemv_dense": 0, "gemv_batch_sparse": 0}, res
