"""Galois rotations and HECTR's he_gemv at the benchmark ring sizes, product
(libgpqhe.so on MI355X) vs oracle, bit for bit.

HECTR's hot call is he_gemv (reference src/hempc.c:257-259) with `slots`
rotation keys from he_genrk (src/ctr.c:521,526-532).  test_gpu_parity.py
covers them at n <= 2^13; here they run at N=2^16, L=8 on both prime sets of
the headline (bench51: every modulus below 2^51, the FP64 path; bench_d2: the
60-bit q0 / P set, whose q0 and P slots take the integer form of the
inner-product kernel and the mixed-set ModUp / ModDown) and at config 5's
N=2^17, L=12 on both (c5f, c5), with 16 slots (HECTR's own count) and 64; the
batch entry points also at n = 2^13 / 2^15 on mixed sets (c1, hyb, c15):

* he_genrk: a subset of the rotation keys, residue by residue;
* he_rot by 1, 3 and slots - 1;
* he_gemv with a matrix that has zero diagonals (skipped) and non-zero ones;
* he_gemv_batch / he_rot_batch over independent ciphertexts sharing M and
  the keys (the batched, key-stationary path; bench.py's gemv leg).

Decoded results are checked against numpy (np.roll, M @ z).
"""
import numpy as np
import pytest

from tests.test_gpu_parity import PARAMS, same

pytestmark = pytest.mark.gpu


def init_slots(oracle, product, name, slots, seed=77):
    kind, kw = PARAMS[name]
    kw = dict(kw, slots=slots)
    for e in (oracle, product):
        e.init_params(**kw)
        e.set_seed(seed)
    assert oracle.primes == product.primes


def rot_keys(e):
    pk, sk = e.pk(), e.sk()
    e.keypair(pk, sk)
    rk = e.evks(e.slots)
    e.genrk(rk, sk)
    return pk, sk, rk


def sample_matrix(s, seed):
    """Dense real/complex entries with every third diagonal zero (the
    all-zero diagonals are skipped by both engines)."""
    rng = np.random.default_rng(seed)
    M = rng.uniform(-1, 1, (s, s)) + 1j * rng.uniform(-1, 1, (s, s))
    M *= (np.add.outer(-np.arange(s), np.arange(s)) % s % 3 != 2)
    return M


@pytest.mark.parametrize("name,slots", [("bench51", 16), ("bench51", 64), ("bench_d2", 16), ("c5f", 16),
                                        ("c5f", 64), ("c5", 16)])
def test_genrk_rot_gemv_large_n(oracle, product, name, slots):
    init_slots(oracle, product, name, slots)
    s = slots
    ko, kp = rot_keys(oracle), rot_keys(product)
    for r in sorted({1, 2, 3, s // 2, s - 1}):
        same(oracle, product, ko[2][r], kp[2][r])
    rng = np.random.default_rng(s)
    z = rng.uniform(-1, 1, s) + 1j * rng.uniform(-1, 1, s)
    M = sample_matrix(s, 5)
    res = {}
    for e, (pk, sk, rk) in ((oracle, ko), (product, kp)):
        x = e.encrypt(z, pk)
        out = {}
        for r in (1, 3, s - 1):
            c = e.ct()
            e.rot(c, x, r, rk)
            out[f"rot{r}"] = c
        c = e.ct()
        e.gemv(c, M.ravel(), x, rk)
        out["gemv"] = c
        res[e.name] = out
    for k in res["oracle"]:
        same(oracle, product, res["oracle"][k], res["product"][k])
    sk = kp[1]
    for r in (1, 3, s - 1):
        got = product.decrypt(res["product"][f"rot{r}"], sk)
        assert np.abs(got - np.roll(z, -r)).max() < 1e-6, r
    got = product.decrypt(res["product"]["gemv"], sk)
    assert np.abs(got - M @ z).max() < 1e-6 * max(1.0, np.abs(M @ z).max())
    for e, k in ((oracle, ko), (product, kp)):
        e.free_evks(k[2])


def encrypt_batch(e, pk, zs, nlimbs=None):
    return np.concatenate([e.export(e.encrypt(z, pk, nlimbs=nlimbs)).ravel() for z in zs])


def run_batch(oracle, product, ko, kp, fn, host_in, out_words, *args):
    """fn(out, *args) on both engines: args hold the input array where the
    string "IN" stands; returns (oracle output, product output)."""
    import torch
    out_o = np.full(out_words, 7, dtype=np.uint64)
    a_o = [host_in.ctypes.data if a == "IN" else a for a in args]
    getattr(oracle.lib, fn)(out_o.ctypes.data, *a_o, ko)
    din = torch.from_numpy(host_in.view(np.int64)).cuda()
    dout = torch.full((out_words,), 7, dtype=torch.int64, device="cuda")
    torch.cuda.synchronize()
    a_p = [din.data_ptr() if a == "IN" else a for a in args]
    getattr(product.lib, fn)(dout.data_ptr(), *a_p, kp)
    product.sync()
    got = dout.cpu().numpy().view(np.uint64)
    return out_o, got


@pytest.mark.parametrize("name,slots,cnt,lvl", [("bench51", 16, 3, 8), ("bench51", 16, 17, 8), ("bench51", 64, 5, 8),
                                                ("bench51", 16, 4, 5), ("bench_d2", 16, 3, 8), ("bench_d2", 16, 17, 8),
                                                ("bench_d2", 16, 4, 5), ("c5f", 16, 3, 12), ("c5f", 64, 2, 12),
                                                ("c5", 16, 2, 12), ("c14", 16, 9, 6), ("c15", 16, 5, 6), ("i14", 16, 3, 6),
                                                ("k5", 16, 3, 4),
                                                ("c1", 16, 3, 4), ("hyb", 16, 3, 5)])
def test_gemv_rot_batch(oracle, product, name, slots, cnt, lvl):
    """he_gemv_batch and he_rot_batch over `cnt` real encryptions at level
    lvl (below the top: a partial digit at lvl 5 of bench51), every output
    residue against the oracle, decoded against M @ z and np.roll."""
    init_slots(oracle, product, name, slots, seed=31)
    s, n = slots, product.n
    ko, kp = rot_keys(oracle), rot_keys(product)
    rng = np.random.default_rng(cnt + s)
    zs = rng.uniform(-1, 1, (cnt, s)) + 1j * rng.uniform(-1, 1, (cnt, s))
    M = sample_matrix(s, 9)
    Mc = np.ascontiguousarray(M.ravel(), dtype=np.complex128)
    host = encrypt_batch(product, kp[0], zs, nlimbs=lvl)
    want, got = run_batch(oracle, product, ko[2], kp[2], "he_gemv_batch", host,
                          cnt * 2 * (lvl - 1) * n, Mc.ctypes.data, "IN", cnt, lvl)
    assert np.array_equal(got, want), f"gemv: {np.count_nonzero(got != want)} residues differ"
    sk, delta = kp[1], product.info.delta
    for i in range(cnt):
        ct = product.ct()
        product.import_(ct, got.reshape(cnt, -1)[i], lvl - 1, scale=delta)
        dz = product.decrypt(ct, sk)
        product.free(ct)
        assert np.abs(dz - M @ zs[i]).max() < 1e-6 * max(1.0, np.abs(M @ zs[i]).max()), i
    for r in (1, s - 1):
        want, got = run_batch(oracle, product, ko[2], kp[2], "he_rot_batch", host,
                              cnt * 2 * lvl * n, "IN", cnt, lvl, r)
        assert np.array_equal(got, want), f"rot {r}: {np.count_nonzero(got != want)} residues differ"
        ct = product.ct()
        product.import_(ct, got.reshape(cnt, -1)[cnt - 1], lvl, scale=delta)
        dz = product.decrypt(ct, sk)
        product.free(ct)
        assert np.abs(dz - np.roll(zs[cnt - 1], -r)).max() < 1e-6
    for e, k in ((oracle, ko), (product, kp)):
        e.free_evks(k[2])


@pytest.mark.parametrize("name", ["bench51", "bench_d2"])
@pytest.mark.parametrize("diags", [(0, 5), (1, 2, 3, 4, 5), (0, 3, 6, 9, 12, 15), (2, 9, 14)])
def test_gemv_batch_few_diagonals(oracle, product, name, diags):
    """he_gemv_batch with a handful of non-zero diagonals: launches of fewer
    than 4 diagonals (the c0 term in the digit kernel) and of 5-6 (its own
    pass, the next source block requested at the last diagonal), with and
    without the identity, on FP64 and mixed prime sets, against the oracle and
    M @ z."""
    init_slots(oracle, product, name, 16, seed=57)
    s, n, lvl, cnt = 16, product.n, 8, 5
    ko, kp = rot_keys(oracle), rot_keys(product)
    rng = np.random.default_rng(len(diags))
    zs = rng.uniform(-1, 1, (cnt, s)) + 1j * rng.uniform(-1, 1, (cnt, s))
    M = rng.uniform(-1, 1, (s, s)) + 1j * rng.uniform(-1, 1, (s, s))
    M *= np.isin(np.add.outer(-np.arange(s), np.arange(s)) % s, diags)
    Mc = np.ascontiguousarray(M.ravel(), dtype=np.complex128)
    host = encrypt_batch(product, kp[0], zs, nlimbs=lvl)
    want, got = run_batch(oracle, product, ko[2], kp[2], "he_gemv_batch", host, cnt * 2 * (lvl - 1) * n,
                          Mc.ctypes.data, "IN", cnt, lvl)
    assert np.array_equal(got, want), f"gemv: {np.count_nonzero(got != want)} residues differ"
    sk, delta = kp[1], product.info.delta
    ct = product.ct()
    product.import_(ct, got.reshape(cnt, -1)[cnt - 1], lvl - 1, scale=delta)
    dz = product.decrypt(ct, sk)
    product.free(ct)
    assert np.abs(dz - M @ zs[cnt - 1]).max() < 1e-6 * max(1.0, np.abs(M @ zs[cnt - 1]).max())
    for e, k in ((oracle, ko), (product, kp)):
        e.free_evks(k[2])


@pytest.mark.parametrize("switch", ["GPQHE_DN_PRE", "GPQHE_DN_S79"])
@pytest.mark.parametrize("name", ["bench51", "bench_d2"])
def test_gemv_rot_batch_dn_pre_off(oracle, product, monkeypatch, name, switch):
    """GPQHE_DN_PRE=0: the ModDown of he_gemv_batch / he_rot_batch on the
    generic column kernel with the scale after its inverse column pass,
    instead of the pre-scaled row pass + dn_colsf form; GPQHE_DN_S79=0: the
    pre-scaled form on the 256 x 256 tiling instead of 128 x 512
    -- the same residues as the oracle either way."""
    init_slots(oracle, product, name, 16, seed=43)
    s, n, lvl, cnt = 16, product.n, 8, 3
    ko, kp = rot_keys(oracle), rot_keys(product)
    rng = np.random.default_rng(7)
    zs = rng.uniform(-1, 1, (cnt, s)) + 1j * rng.uniform(-1, 1, (cnt, s))
    Mc = np.ascontiguousarray(sample_matrix(s, 5).ravel(), dtype=np.complex128)
    host = encrypt_batch(product, kp[0], zs, nlimbs=lvl)
    monkeypatch.setenv(switch, "0")
    want, got = run_batch(oracle, product, ko[2], kp[2], "he_gemv_batch", host, cnt * 2 * (lvl - 1) * n,
                          Mc.ctypes.data, "IN", cnt, lvl)
    assert np.array_equal(got, want), f"gemv: {np.count_nonzero(got != want)} residues differ"
    want, got = run_batch(oracle, product, ko[2], kp[2], "he_rot_batch", host, cnt * 2 * lvl * n, "IN", cnt, lvl, 2)
    assert np.array_equal(got, want), f"rot: {np.count_nonzero(got != want)} residues differ"
    for e, k in ((oracle, ko), (product, kp)):
        e.free_evks(k[2])


def test_gemv_rot_batch_chunks_and_empty(oracle, product, monkeypatch):
    """The batch path's chunk loop (GPQHE_GEMV_CHUNK=2: 5 ciphertexts as
    2 + 2 + 1, the workspace and orbit table per chunk) against the oracle, and
    empty batches (count 0) that leave the output untouched."""
    import torch
    init_slots(oracle, product, "bench51", 16, seed=41)
    s, n, lvl, cnt = 16, product.n, 8, 5
    ko, kp = rot_keys(oracle), rot_keys(product)
    rng = np.random.default_rng(5)
    zs = rng.uniform(-1, 1, (cnt, s)) + 1j * rng.uniform(-1, 1, (cnt, s))
    Mc = np.ascontiguousarray(sample_matrix(s, 3).ravel(), dtype=np.complex128)
    host = encrypt_batch(product, kp[0], zs, nlimbs=lvl)
    monkeypatch.setenv("GPQHE_GEMV_CHUNK", "2")
    want, got = run_batch(oracle, product, ko[2], kp[2], "he_gemv_batch", host, cnt * 2 * (lvl - 1) * n,
                          Mc.ctypes.data, "IN", cnt, lvl)
    assert np.array_equal(got, want), f"gemv: {np.count_nonzero(got != want)} residues differ"
    want, got = run_batch(oracle, product, ko[2], kp[2], "he_rot_batch", host, cnt * 2 * lvl * n, "IN", cnt, lvl, 3)
    assert np.array_equal(got, want), f"rot: {np.count_nonzero(got != want)} residues differ"
    din = torch.from_numpy(host.view(np.int64)).cuda()
    dout = torch.full((2 * lvl * n,), 7, dtype=torch.int64, device="cuda")
    torch.cuda.synchronize()
    product.lib.he_gemv_batch(dout.data_ptr(), Mc.ctypes.data, din.data_ptr(), 0, lvl, kp[2])
    product.lib.he_rot_batch(dout.data_ptr(), din.data_ptr(), 0, lvl, 3, kp[2])
    product.sync()
    assert bool((dout == 7).all())
    for e, k in ((oracle, ko), (product, kp)):
        e.free_evks(k[2])


def test_gemv_generic_path():
    """GPQHE_GEMV_WIN=0 (read once per process, so in a child process): the
    round-4 generic kernels (one ciphertext at a time, the baseline of
    profiles/r5_gemv_baseline_generic*.json) stay bit-exact against the
    oracle at the bench's shape."""
    import json
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, GPQHE_GEMV_WIN="0")
    r = subprocess.run([sys.executable, os.path.join(root, "tests", "gemv_switch_worker.py")], env=env, cwd=root,
                       capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-3000:]
    res = json.loads([x for x in r.stdout.splitlines() if x.startswith("{")][-1])
    assert res == {"gemv_batch": 0, "rot_batch": 0}, res
