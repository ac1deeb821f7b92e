"""Generate tests/golden/model_vectors.json from the pure-Python model only
(no oracle, no product): prime/root selection rule, NTT by definition,
exact rescale.  Run: python tests/make_golden.py"""
import json
import os
import random

import ckks_model as M

HERE = os.path.dirname(os.path.abspath(__file__))


def pick(bits, two_n, used):
    top = 1 << bits
    c = (top // two_n) * two_n + 1
    while c >= top:
        c -= two_n
    while c > top >> 1:
        if c not in used and M.is_prime(c):
            return c
        c -= two_n
    raise ValueError("no prime")


def psi_of(q, n):
    h = 2
    while True:
        p = pow(h, (q - 1) // (2 * n), q)
        if pow(p, n, q) == q - 1:
            return p
        h += 1


def main():
    rnd = random.Random(20261015)
    out = {"ntt": [], "rescale": []}
    for logn, bits in ((4, 40), (6, 40), (8, 50)):
        n = 1 << logn
        q = pick(bits, 2 * n, [])
        psi = psi_of(q, n)
        x = [rnd.randrange(q) for _ in range(n)]
        out["ntt"].append({"logn": logn, "bits": bits, "q": q, "psi": psi, "input": x,
                           "ntt": M.ntt_eval(x, q, psi)})
    logn = 5
    n = 1 << logn
    used = []
    for b in (40, 36, 36):
        used.append(pick(b, 2 * n, used))
    inp, res = [], []
    coef = [[[rnd.randrange(q) for _ in range(n)] for q in used] for _ in range(2)]
    for p in range(2):
        for i in range(3):
            inp.extend(coef[p][i])
    for p in range(2):
        outp = [[0] * n for _ in range(2)]
        for k in range(n):
            X, _ = M.crt([coef[p][i][k] for i in range(3)], used)
            Y = (X - X % used[2]) // used[2]
            for i in range(2):
                outp[i][k] = Y % used[i]
        res.extend(outp[0] + outp[1])
    out["rescale"].append({"logn": logn, "primes": used, "input": inp, "output": res})
    with open(os.path.join(HERE, "golden", "model_vectors.json"), "w") as f:
        json.dump(out, f)


if __name__ == "__main__":
    main()
