"""Small-N step sequences shared by the GPU parity tests and the switch worker.

Each function drives one engine (product or oracle) through a sequence of
HECTR-style control-step calls and returns every exported object and decoded
vector in call order; the tests compare the two engines' lists bit for bit.
The sequences follow the reference's regulator step: encode + encrypt the
state (src/ctr.c:461-480), he_sub x2, he_gemv x2, he_add / he_neg
(src/hempc.c:253-266), decrypt + decode (src/ctr.c:486-490).
"""
import numpy as np

PARAMS_REF = dict(logn=12, logq=109, slots=16, log_delta=50)  # src/ctr.c:514-518


def keys(e, rot=True):
    pk, sk = e.pk(), e.sk()
    e.keypair(pk, sk)
    rk = None
    if rot:
        rk = e.evks(e.slots)
        e.genrk(rk, sk)
    return pk, sk, rk


def speculative_noise(e, seed=1234, rng_seed=9):
    """Steps of 5 encryptions (HECTR's), then 3 (a prefix of the speculated
    streams), 6 (more than speculated), one with a live plaintext, one at a
    lower level, a reseed between steps (api.cpp SpecNoise)."""
    e.init(**PARAMS_REF)
    e.set_seed(seed)
    rng = np.random.default_rng(rng_seed)
    plan = [5, 5, 3, 6, "live", "lvl1", "reseed", 5, 5]
    zs = [[rng.uniform(-1, 1, e.slots) + 0j for _ in range(6)] for _ in plan]
    pk, sk, _ = keys(e, rot=False)
    res = []
    for kind, zz in zip(plan, zs):
        if kind == "reseed":
            e.set_seed(77)
            continue
        cnt = kind if isinstance(kind, int) else 2
        lvl = 1 if kind == "lvl1" else e.L
        pts, cts = [], []
        for z in zz[:cnt]:
            pt = e.pt()
            e.ecd_ex(pt, z, e.slots, e.info.delta, lvl)
            pts.append(pt)
        for pt in pts:
            ct = e.ct()
            e.enc_pk(ct, pt, pk)
            cts.append(ct)
        if kind == "live":
            res.append(e.export(pts[0]))
        for pt in pts:
            e.free(pt)
        d = e.ct()
        e.sub(d, cts[0], cts[1])
        res += [e.export(x) for x in cts + [d]]
        res.append(e.decrypt(d, sk))  # he_dcd: the next step's noise is launched behind it
        for x in cts + [d]:
            e.free(x)
    return res


def queued_differences(e, seed=1234, rng_seed=31):
    """HECTR's regulator step repeated (api.cpp ew_lazy_sub: from the second
    step on the subs stay queued and gemv_inner_kernel forms the differences
    from their operands).  Variants per step: the differences freed unread,
    read back after the gemvs, an operand of a sub overwritten after the
    gemvs, an in-place he_gemv(x, M, x), a gemv whose output is an operand of
    the queued sub, and a non-speculated step (four encryptions)."""
    e.init(**PARAMS_REF)
    e.set_seed(seed)
    rng = np.random.default_rng(rng_seed)
    s = e.slots
    M1 = (rng.uniform(-1, 1, (s, s)) + 0j).astype(np.complex128)
    M2 = (rng.uniform(-1, 1, (s, s)) + 0j).astype(np.complex128)
    plan = ["free", "free", "read", "free", "clobber", "free", "inplace", "free", "ycts", "free", "four", "free",
            "free"]
    zs = [[rng.uniform(-1, 1, s) + 0j for _ in range(5)] for _ in plan]
    pk, sk, rk = keys(e, rot=True)
    res = []
    for kind, zz in zip(plan, zs):
        cnt = 4 if kind == "four" else 5
        cts = [e.encrypt(z, pk) for z in zz[:cnt]]
        xd, ud = e.ct(), e.ct()
        e.sub(xd, cts[0], cts[1])
        e.sub(ud, cts[2], cts[3])
        if kind == "inplace":  # he_gemv(x, M, x): the output is the queued sub's output
            ya = xd
        elif kind == "ycts":  # the output is an operand of the queued sub
            ya = cts[0]
        else:
            ya = e.ct()
        yb = e.ct()
        e.gemv(ya, M1.ravel(), xd, rk)
        e.gemv(yb, M2.ravel(), ud, rk)
        du = e.ct()
        e.add(du, ya, yb)
        e.neg(du)
        if kind == "read":
            res += [e.export(xd), e.export(ud)]
        if kind == "clobber":
            e.add(cts[0], cts[0], cts[1])  # an operand of the first sub
            res.append(e.export(cts[0]))
        res += [e.export(ya), e.export(yb), e.export(du)]
        for x in (xd, ud, yb) + (() if kind in ("inplace", "ycts") else (ya,)):
            e.free(x)
        res.append(e.decrypt(du, sk))
        for x in cts + [du]:
            e.free(x)
    return res


def rekeyed_steps(e, seed=1234, rng_seed=41):
    """The regulator step with the public key changing between speculative
    steps (api.cpp SpecModup is keyed on the public key's block): two steps
    on key A; A freed and a new key C generated (its block may be A's); steps
    on C; then keys B and C alternating step by step."""
    e.init(**PARAMS_REF)
    e.set_seed(seed)
    rng = np.random.default_rng(rng_seed)
    s = e.slots
    M1 = (rng.uniform(-1, 1, (s, s)) + 0j).astype(np.complex128)
    M2 = (rng.uniform(-1, 1, (s, s)) + 0j).astype(np.complex128)
    ks = {"A": keys(e), "B": keys(e)}
    plan = ["A", "A", "newC", "C", "C", "B", "C", "B", "C", "C"]
    zs = [[rng.uniform(-1, 1, s) + 0j for _ in range(5)] for _ in plan]
    res = []
    for kind, zz in zip(plan, zs):
        if kind == "newC":
            pk, sk, rk = ks.pop("A")
            e.free(pk)
            e.free(sk)
            e.free_evks(rk)
            ks["C"] = keys(e)
            kind = "C"
        pk, sk, rk = ks[kind]
        cts = [e.encrypt(z, pk) for z in zz]
        xd, ud, ya, yb, du = e.ct(), e.ct(), e.ct(), e.ct(), e.ct()
        e.sub(xd, cts[0], cts[1])
        e.sub(ud, cts[2], cts[3])
        e.gemv(ya, M1.ravel(), xd, rk)
        e.gemv(yb, M2.ravel(), ud, rk)
        e.add(du, ya, yb)
        e.neg(du)
        res += [e.export(ya), e.export(yb), e.export(du)]
        for x in (xd, ud, ya, yb):
            e.free(x)
        res.append(e.decrypt(du, sk))
        for x in cts + [du]:
            e.free(x)
    return res


def speculative_gemvs(e, seed=1234, rng_seed=53, plan=None):
    """HECTR's step with its own call order (all five encodes, all five
    encryptions, the plaintexts freed: src/ctr.c:461-480, which starts the
    early combine and, from the third step on, the speculated gemvs of the
    last step's pattern, api.cpp SpecGemv), and steps where the speculation
    must not be taken: a gemv matrix that changed, the subtraction's operands
    swapped, an encryption overwritten before its he_sub, the gemvs in the
    other order, the rotation keys regenerated in place, and one gemv only."""
    e.init(**PARAMS_REF)
    e.set_seed(seed)
    rng = np.random.default_rng(rng_seed)
    s = e.slots
    M1 = (rng.uniform(-1, 1, (s, s)) + 0j).astype(np.complex128)
    M2 = (rng.uniform(-1, 1, (s, s)) + 0j).astype(np.complex128)
    M3 = (rng.uniform(-1, 1, (s, s)) + 0j).astype(np.complex128)
    plan = plan or ["same", "same", "same", "newM", "same", "swap", "same", "clobber", "same", "order", "same",
                    "regen", "same", "one", "same", "same"]
    zs = [[rng.uniform(-1, 1, s) + 0j for _ in range(5)] for _ in plan]
    pk, sk, rk = keys(e, rot=True)
    res, keep = [], []
    for kind, zz in zip(plan, zs):
        if kind == "regen":
            e.genrk(rk, sk)
        pts = []
        for z in zz:
            pt = e.pt()
            e.ecd(pt, z)
            pts.append(pt)
        cts = []
        for pt in pts:
            ct = e.ct()
            e.enc_pk(ct, pt, pk)
            cts.append(ct)
        for pt in pts:
            e.free(pt)
        if kind == "clobber":
            e.add(cts[1], cts[1], cts[4])
        xd, ud, ya, yb, du = e.ct(), e.ct(), e.ct(), e.ct(), e.ct()
        if kind == "swap":
            e.sub(xd, cts[2], cts[1])
        else:
            e.sub(xd, cts[1], cts[2])
        e.sub(ud, cts[3], cts[4])
        Ma = M3 if kind == "newM" else M1
        if kind == "order":
            e.gemv(yb, M2.ravel(), ud, rk)
            e.gemv(ya, Ma.ravel(), xd, rk)
        elif kind == "one":
            e.gemv(ya, Ma.ravel(), xd, rk)
            e.copy_ct(yb, ya)
        elif kind == "realias":
            # the speculated result freed and its block (likely) handed to a
            # gemv that is not speculated (another matrix), whose queued launch
            # writes it before the tail reads it (SpecDcd must not replay)
            e.gemv(ya, Ma.ravel(), xd, rk)
            e.gemv(yb, M2.ravel(), ud, rk)
            e.free(ya)
            ya = e.ct()
            e.gemv(ya, M3.ravel(), ud, rk)
        else:
            e.gemv(ya, Ma.ravel(), xd, rk)
            e.gemv(yb, M2.ravel(), ud, rk)
        e.add(du, ya, yb)
        e.neg(du)
        e.add(du, du, cts[0])
        # (exported after the last step: an export runs every queue and
        # forgets the speculation records, as any non-queued call does)
        keep += [ya, yb, du]
        for x in (xd, ud):
            e.free(x)
        res.append(e.decrypt(du, sk))
        for x in cts:
            e.free(x)
    res += [e.export(x) for x in keep]
    return res


SEQUENCES = {"speculative_noise": speculative_noise, "queued_differences": queued_differences,
             "rekeyed_steps": rekeyed_steps, "speculative_gemvs": speculative_gemvs}


def mismatches(a, b):
    """Indices where two sequence results differ (a length mismatch is one)."""
    if len(a) != len(b):
        return [-1]
    return [i for i, (x, y) in enumerate(zip(a, b)) if not np.array_equal(x, y)]
