"""Independent pure-Python big-integer model of the arithmetic the engine
claims to compute (test infrastructure only).

Nothing here shares code with the oracle (C) or the product (HIP): NTTs are
evaluated from the definition, polynomials are multiplied by schoolbook
negacyclic convolution, RNS values are recombined with exact Python
integers.  Used to pin the oracle (tests/test_oracle_model.py) and to make
the committed known-answer vectors (tests/make_golden.py).
"""
from __future__ import annotations

import cmath
import math


def brev(x: int, bits: int) -> int:
    r = 0
    for _ in range(bits):
        r = (r << 1) | (x & 1)
        x >>= 1
    return r


def is_prime(n: int) -> bool:
    if n < 2:
        return False
    for p in (2, 3, 5, 7, 11, 13, 17, 19, 23, 29, 31, 37):
        if n % p == 0:
            return n == p
    d, r = n - 1, 0
    while d % 2 == 0:
        d //= 2
        r += 1
    for a in (2, 3, 5, 7, 11, 13, 17, 19, 23, 29, 31, 37):
        x = pow(a, d, n)
        if x in (1, n - 1):
            continue
        for _ in range(r - 1):
            x = x * x % n
            if x == n - 1:
                break
        else:
            return False
    return True


def ntt_eval(a, q, psi):
    """A[k] = a(psi^(2 brev(k) + 1)) mod q (bit-reversed evaluation order)."""
    n = len(a)
    logn = n.bit_length() - 1
    out = []
    for k in range(n):
        x = pow(psi, 2 * brev(k, logn) + 1, q)
        acc, p = 0, 1
        for c in a:
            acc = (acc + c * p) % q
            p = p * x % q
        out.append(acc)
    return out


def negacyclic_mul(a, b, q):
    n = len(a)
    out = [0] * n
    for i, x in enumerate(a):
        if not x:
            continue
        for j, y in enumerate(b):
            k = i + j
            if k < n:
                out[k] = (out[k] + x * y) % q
            else:
                out[k - n] = (out[k - n] - x * y) % q
    return out


def automorphism(a, g, q):
    """a(X) -> a(X^g) in Z_q[X]/(X^n + 1)."""
    n = len(a)
    out = [0] * n
    for j, c in enumerate(a):
        e = j * g % (2 * n)
        if e < n:
            out[e] = (out[e] + c) % q
        else:
            out[e - n] = (out[e - n] - c) % q
    return out


def crt(residues, primes):
    """Exact value in [0, prod primes)."""
    Q = 1
    for p in primes:
        Q *= p
    x = 0
    for r, p in zip(residues, primes):
        Qi = Q // p
        x += r * Qi * pow(Qi, -1, p)
    return x % Q, Q


def center(x, Q):
    return x - Q if x > Q // 2 else x


def special_decode(u):
    """z_j = sum_k u_k xi^(k 5^j), xi = exp(2 pi i / 4s)."""
    s = len(u)
    M = 4 * s
    return [sum(u[k] * cmath.exp(2j * math.pi * k * pow(5, j, M) / M) for k in range(s)) for j in range(s)]


def special_encode(z):
    s = len(z)
    M = 4 * s
    return [sum(z[j] * cmath.exp(-2j * math.pi * k * pow(5, j, M) / M) for j in range(s)) / s for k in range(s)]


def encode_coeffs(z, n, scale):
    """Coefficients of the CKKS encoding of z (len s) at `scale`."""
    s = len(z)
    u = special_encode(z)
    gap = n // (2 * s)
    coef = [0] * n
    for k in range(s):
        coef[k * gap] = round(u[k].real * scale)
        coef[(k + s) * gap] = round(u[k].imag * scale)
    return coef
