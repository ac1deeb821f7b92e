"""The CPU oracle pinned against the independent big-integer model
(tests/ckks_model.py) and the committed known-answer vectors
(tests/golden/model_vectors.json).  CPU only."""
import ctypes
import json
import os

import numpy as np
import pytest

import ckks_model as M

HERE = os.path.dirname(os.path.abspath(__file__))


def small_ctx(oracle, logn, nlimbs=2, nspecial=1, dnum=None, slots=None, seed=5, qb=(40, 36, 41)):
    oracle.init_params(logn=logn, nlimbs=nlimbs, nspecial=nspecial, dnum=dnum or nlimbs,
                       slots=slots or (1 << (logn - 1)), q0_bits=qb[0], qi_bits=qb[1], p_bits=qb[2], seed=seed)
    return oracle


@pytest.mark.parametrize("logn", [4, 6, 8, 12, 16])
def test_primes_and_roots(oracle, logn):
    small_ctx(oracle, logn, nlimbs=3, nspecial=2, qb=(60, 50, 60))
    n = 1 << logn
    primes = oracle.primes
    assert len(set(primes)) == len(primes)
    for i, q in enumerate(primes):
        assert M.is_prime(q) and q % (2 * n) == 1
        bits = 60 if i in (0, 3, 4) else 50
        assert q < 1 << bits
        # largest such prime below 2^bits not used earlier in the chain
        c = q + 2 * n
        while c < 1 << bits:
            assert not M.is_prime(c) or c in primes[:i], (i, c)
            c += 2 * n
        psi = oracle.info.psi[i]
        assert pow(psi, n, q) == q - 1


@pytest.mark.parametrize("logn", [4, 5, 7])
def test_ntt_matches_definition(oracle, logn):
    small_ctx(oracle, logn)
    n, L = oracle.n, oracle.L
    x = np.zeros(L * n, dtype=np.uint64)
    oracle.lib.poly_fill_uniform(x.ctypes.data, 1, L, 3)
    src = x.copy()
    oracle.lib.poly_ntt_batch(x.ctypes.data, 1, L)
    for i in range(L):
        q, psi = oracle.primes[i], oracle.info.psi[i]
        want = M.ntt_eval([int(v) for v in src[i * n:(i + 1) * n]], q, psi)
        assert [int(v) for v in x[i * n:(i + 1) * n]] == want
    oracle.lib.poly_intt_batch(x.ctypes.data, 1, L)
    assert np.array_equal(x, src)


def test_ntt_convolution(oracle):
    small_ctx(oracle, 6)
    n = oracle.n
    q = oracle.primes[0]
    rng = np.random.default_rng(1)
    a = rng.integers(0, q, n, dtype=np.uint64)
    b = rng.integers(0, q, n, dtype=np.uint64)
    A, B = a.copy(), b.copy()
    oracle.lib.poly_ntt_batch(A.ctypes.data, 1, 1)
    oracle.lib.poly_ntt_batch(B.ctypes.data, 1, 1)
    C = np.array([int(x) * int(y) % q for x, y in zip(A, B)], dtype=np.uint64)
    oracle.lib.poly_intt_batch(C.ctypes.data, 1, 1)
    want = M.negacyclic_mul([int(v) for v in a], [int(v) for v in b], q)
    assert [int(v) for v in C] == want


def test_golden_vectors(oracle):
    """Known answers produced by the pure-Python model (tests/make_golden.py)."""
    with open(os.path.join(HERE, "golden", "model_vectors.json")) as f:
        gold = json.load(f)
    for case in gold["ntt"]:
        small_ctx(oracle, case["logn"], nlimbs=1, qb=(case["bits"], 36, 41))
        assert oracle.primes[0] == case["q"] and oracle.info.psi[0] == case["psi"]
        x = np.array(case["input"], dtype=np.uint64)
        oracle.lib.poly_ntt_batch(x.ctypes.data, 1, 1)
        assert [int(v) for v in x] == case["ntt"]
    for case in gold["rescale"]:
        small_ctx(oracle, case["logn"], nlimbs=3, qb=(40, 36, 41))
        assert oracle.primes[:3] == case["primes"]
        ct = oracle.ct()
        data = np.array(case["input"], dtype=np.uint64).reshape(2, 3, -1)
        ntt = data.copy()
        oracle.lib.poly_ntt_batch(ntt.ctypes.data, 2, 3)
        oracle.import_(ct, ntt, 3, scale=1.0)
        oracle.rescale(ct)
        out = oracle.export(ct).copy()
        oracle.lib.poly_intt_batch(out.ctypes.data, 2, 2)
        assert out.reshape(-1).tolist() == case["output"]
        oracle.free(ct)


def test_automorphism_and_rotation(oracle):
    """Galois 5^r in the NTT domain equals X -> X^(5^r) on coefficients, and
    he_rot decrypts to the rotated slots (model decryption by exact CRT)."""
    small_ctx(oracle, 6, nlimbs=2, slots=8, qb=(55, 45, 58))
    n, L = oracle.n, oracle.L
    pk, sk = oracle.pk(), oracle.sk()
    oracle.keypair(pk, sk)
    rk = oracle.evks(8)
    oracle.genrk(rk, sk)
    rng = np.random.default_rng(4)
    z = rng.uniform(-1, 1, 8) + 1j * rng.uniform(-1, 1, 8)
    ct = oracle.encrypt(z, pk)
    out = oracle.ct()
    oracle.rot(out, ct, 3, rk)
    s = oracle.export(sk)[0]
    c = oracle.export(out).copy()
    primes = oracle.primes[:L]
    # model decryption: m = c0 + c1 s in the NTT domain, then inverse NTT by
    # the definition (solve via the oracle's INTT, checked in another test)
    m = np.zeros((L, n), dtype=np.uint64)
    for i, q in enumerate(primes):
        m[i] = [(int(a) + int(b) * int(t)) % q for a, b, t in zip(c[0, i], c[1, i], s[i])]
    oracle.lib.poly_intt_batch(m.ctypes.data, 1, L)
    coef = [M.center(*M.crt([int(m[i, k]) for i in range(L)], primes)) for k in range(n)]
    gap = n // 16
    u = [complex(coef[k * gap], coef[(k + 8) * gap]) / out.scale for k in range(8)]
    got = np.array(M.special_decode(u))
    assert np.abs(got - np.roll(z, -3)).max() < 1e-6
    # and the NTT-domain automorphism against the coefficient definition
    x = np.zeros(n, dtype=np.uint64)
    oracle.lib.poly_fill_uniform(x.ctypes.data, 1, 1, 8)
    q = primes[0]
    g = pow(5, 3, 2 * n)
    y = M.automorphism([int(v) for v in x], g, q)
    X, Y = x.copy(), np.array(y, dtype=np.uint64)
    oracle.lib.poly_ntt_batch(X.ctypes.data, 1, 1)
    oracle.lib.poly_ntt_batch(Y.ctypes.data, 1, 1)
    logn = n.bit_length() - 1
    perm = [M.brev((((2 * M.brev(k, logn) + 1) * g) % (2 * n) - 1) // 2, logn) for k in range(n)]
    assert all(int(Y[k]) == int(X[perm[k]]) for k in range(n))


def test_encode_matches_model(oracle):
    small_ctx(oracle, 7, nlimbs=2, slots=16, qb=(55, 45, 58))
    rng = np.random.default_rng(9)
    z = rng.uniform(-3, 3, 16) + 1j * rng.uniform(-3, 3, 16)
    pt = oracle.pt()
    oracle.ecd_ex(pt, z, 16, 2.0 ** 30, 2)
    m = oracle.export(pt)[0].copy()
    oracle.lib.poly_intt_batch(m.ctypes.data, 1, 2)
    want = M.encode_coeffs(list(z), oracle.n, 2.0 ** 30)
    for i, q in enumerate(oracle.primes[:2]):
        assert [int(v) for v in m[i]] == [c % q for c in want]
    zz = oracle.dcd(pt, 16)
    assert np.abs(zz - z).max() < 1e-8


def test_rescale_is_exact_floor_division(oracle):
    """he_rescale output = (X - X mod q_top) / q_top on every coefficient."""
    small_ctx(oracle, 5, nlimbs=3, qb=(40, 36, 41))
    n, primes = oracle.n, oracle.primes[:3]
    rng = np.random.default_rng(2)
    coef = rng.integers(0, 2 ** 62, (2, 3, n), dtype=np.uint64)
    for i, q in enumerate(primes):
        coef[:, i] %= np.uint64(q)
    ntt = coef.copy()
    oracle.lib.poly_ntt_batch(ntt.ctypes.data, 2, 3)
    ct = oracle.ct()
    oracle.import_(ct, ntt, 3, scale=2.0 ** 36)
    oracle.rescale(ct)
    out = oracle.export(ct).copy()
    oracle.lib.poly_intt_batch(out.ctypes.data, 2, 2)
    for p in range(2):
        for k in range(n):
            X, _ = M.crt([int(coef[p, i, k]) for i in range(3)], primes)
            Y = (X - X % primes[2]) // primes[2]
            assert [int(out[p, i, k]) for i in range(2)] == [Y % q for q in primes[:2]]


@pytest.mark.parametrize("params", [dict(nlimbs=3, nspecial=1, dnum=3), dict(nlimbs=4, nspecial=2, dnum=2)])
def test_mul_relin_model_decrypt(oracle, params):
    """ct x ct + relinearization + rescale decrypts (exact CRT model) to the
    slot-wise product; exercises ModUp/ModDown with alpha = 1 and 2, K = 1, 2."""
    small_ctx(oracle, 6, slots=8, qb=(55, 40, 58), **params)
    pk, sk = oracle.pk(), oracle.sk()
    oracle.keypair(pk, sk)
    rlk = oracle.evk()
    oracle.genrlk(rlk, sk)
    rng = np.random.default_rng(6)
    z1 = rng.uniform(-1, 1, 8) + 1j * rng.uniform(-1, 1, 8)
    z2 = rng.uniform(-1, 1, 8) + 1j * rng.uniform(-1, 1, 8)
    a = oracle.encrypt(z1, pk, slots=8, scale=2.0 ** 40)
    b = oracle.encrypt(z2, pk, slots=8, scale=2.0 ** 40)
    c = oracle.ct()
    oracle.mul_rescale(c, a, b, rlk)
    assert c.nlimbs == params["nlimbs"] - 1
    got = oracle.decrypt(c, sk, slots=8)
    assert np.abs(got - z1 * z2).max() < 1e-6
