"""Product (libgpqhe.so on MI355X) vs oracle (CPU restatement): bit-exact
parity of every he_* operation on identical seeded inputs.

Parameter sets:
  ref   : HECTR's own hectx_init(logn=12, q=2^109, slots=16, Delta=2^50)
          (reference src/ctr.c:514-518) -> n=4096, L=2, K=1, dnum=2
  c1    : config 1 sizes, n=2^13, L=4 (dnum=4)
  hyb   : n=2^13, L=5, K=2, dnum=3 (digits {0,1} {2,3} {4}: exercises the
          fast basis conversion with alpha > 1, K > 1 and a partial digit;
          P = 2^118 exceeds every digit modulus, as hybrid switching needs)
  bench : config 2/3 sizes, n=2^16, L=8, K=1, dnum=8
  bench_d2: the bench's own parameters, n=2^16, L=8, K=4, dnum=2
  c5    : config 5 sizes, n=2^17, L=12, K=4, dnum=3 (the multi-GPU config)
  bench51: the bench shape with every prime below 2^51, so every NTT and the
          key inner product run on the FP64 path
  c17   : n=2^17, L=8, K=4, dnum=2, primes < 2^51 (the 2^17 fused path with the
          key-stationary two-digit inner product)
  c14/c15: n=2^14 (all primes < 2^51) and n=2^15 (60-bit q0/P: mixed FP64 and
          integer limbs), L=6, K=3, dnum=2 -- the other fused tilings
  a5    : n=2^13, L=5, dnum=1 (one 5-limb digit), K=4
Integer results must match exactly; decoded values are compared with the
closed-loop tolerance of the CSTR test (1e-6 relative, reference achieves
1e-11).
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

PARAMS = {
    "ref": ("init", dict(logn=12, logq=109, slots=16, log_delta=50)),
    "c1": ("params", dict(logn=13, nlimbs=4, slots=64, q0_bits=60, qi_bits=50, p_bits=60)),
    "hyb": ("params", dict(logn=13, nlimbs=5, nspecial=2, dnum=3, slots=32, q0_bits=58, qi_bits=45,
                           p_bits=59)),
    "bench": ("params", dict(logn=16, nlimbs=8, slots=64, q0_bits=60, qi_bits=50, p_bits=60)),
    "bench_d2": ("params", dict(logn=16, nlimbs=8, nspecial=4, dnum=2, slots=64, q0_bits=60, qi_bits=50,
                                p_bits=60)),
    "c5": ("params", dict(logn=17, nlimbs=12, nspecial=4, dnum=3, slots=64, q0_bits=60, qi_bits=50, p_bits=60)),
    # config 5 at the headline's prime sizes (every modulus below 2^51: the
    # all-FP64 three-digit split key switch), bench.py's config5 value
    "c5f": ("params", dict(logn=17, nlimbs=12, nspecial=4, dnum=3, slots=64, q0_bits=51, qi_bits=50, p_bits=51)),
    "bench51": ("params", dict(logn=16, nlimbs=8, nspecial=4, dnum=2, slots=64, q0_bits=51, qi_bits=50,
                               p_bits=51)),
    "c17": ("params", dict(logn=17, nlimbs=8, nspecial=4, dnum=2, slots=64, q0_bits=51, qi_bits=50, p_bits=51)),
    # the remaining fused-path tilings: n=2^14 (64 x 256 columns, 128-element
    # rows) and n=2^15 (128 x 256 columns, 256-element rows)
    "c14": ("params", dict(logn=14, nlimbs=6, nspecial=3, dnum=2, slots=64, q0_bits=51, qi_bits=48, p_bits=51)),
    "c15": ("params", dict(logn=15, nlimbs=6, nspecial=3, dnum=2, slots=64, q0_bits=60, qi_bits=48, p_bits=60)),
    # 61-bit q0 / P: integer moduli of 2^60 and above (the gemv's integer form
    # without its 30-bit-half products)
    "i14": ("params", dict(logn=14, nlimbs=6, nspecial=3, dnum=2, slots=64, q0_bits=61, qi_bits=48, p_bits=61)),
    # five special primes (K > 4: no split key switch / fused ModDown) on an
    # all-FP64 set: the gemv batch path's own ModUp (INTT, gemv_fbc_kernel,
    # NTT) and the generic ModDown
    "k5": ("params", dict(logn=13, nlimbs=4, nspecial=5, dnum=1, slots=64, q0_bits=51, qi_bits=48, p_bits=51)),
    # all-FP64 sets at n=2^13 and 2^15: the FP64 column kernels
    # ks_colsf<6, 8> / dn_colsf<6, .> / ntt2_colsf<6, .> (T = 64) and the
    # n=2^15 split-key-switch forms on every-modulus-below-2^51 primes
    "f13": ("params", dict(logn=13, nlimbs=6, nspecial=3, dnum=2, slots=64, q0_bits=51, qi_bits=48, p_bits=51)),
    "f15": ("params", dict(logn=15, nlimbs=6, nspecial=3, dnum=2, slots=64, q0_bits=51, qi_bits=48, p_bits=51)),
    # one digit of 5 limbs (alpha > 4: the single-target ks_cols_kernel and the
    # streaming ks_rows_kernel), n=2^13, L=5, dnum=1, K=4 (P 240 > 200 bits)
    "a5": ("params", dict(logn=13, nlimbs=5, nspecial=4, dnum=1, slots=64, q0_bits=40, qi_bits=40, p_bits=60)),
    # the headline shape with a 60-bit q0 (HECTR's q = 2^109 = q0 q1 at
    # Delta = 2^50, reference src/ctr.c:514-517) and special primes below 2^51:
    # three digits of 3/3/2 limbs (60 + 100 bits) under P = 4 x 51 bits, so only
    # q0 takes the integer forms
    "m60": ("params", dict(logn=16, nlimbs=8, nspecial=4, dnum=3, slots=64, q0_bits=60, qi_bits=50, p_bits=51)),
}


def init_both(oracle, product, name, seed=1234):
    kind, kw = PARAMS[name]
    for e in (oracle, product):
        if kind == "init":
            e.init(**kw)
        else:
            e.init_params(**kw)
        e.set_seed(seed)
    assert oracle.primes == product.primes
    assert list(oracle.info.psi[:len(oracle.primes)]) == list(product.info.psi[:len(product.primes)])


def keys(e, rot=True):
    pk, sk = e.pk(), e.sk()
    e.keypair(pk, sk)
    rk = None
    if rot:
        rk = e.evks(e.slots)
        e.genrk(rk, sk)
    rlk = e.evk()
    e.genrlk(rlk, sk)
    return pk, sk, rk, rlk


def same(o, p, a, b):
    A, B = o.export(a), p.export(b)
    assert A.shape == B.shape
    bad = np.argwhere(A != B)
    assert bad.size == 0, f"{len(bad)} residues differ, first at {bad[0].tolist()}"


@pytest.mark.parametrize("name", ["ref", "c1", "hyb", "bench"])
def test_keys_encrypt_decrypt(oracle, product, name):
    init_both(oracle, product, name)
    rot = name != "bench"
    ko, kp = keys(oracle, rot), keys(product, rot)
    for a, b in zip(ko, kp):
        if a is None:
            continue
        if hasattr(a, "__len__"):
            for i in range(1, len(a)):
                same(oracle, product, a[i], b[i])
        else:
            same(oracle, product, a, b)
    rng = np.random.default_rng(5)
    z = rng.uniform(-1, 1, oracle.slots) + 1j * rng.uniform(-1, 1, oracle.slots)
    co, cp = oracle.encrypt(z, ko[0]), product.encrypt(z, kp[0])
    same(oracle, product, co, cp)
    zo, zp = oracle.decrypt(co, ko[1]), product.decrypt(cp, kp[1])
    assert np.array_equal(zo, zp)
    assert np.abs(zp - z).max() < 1e-6


@pytest.mark.parametrize("name", ["ref", "c1", "hyb"])
def test_evaluation_ops(oracle, product, name):
    init_both(oracle, product, name)
    ko, kp = keys(oracle), keys(product)
    rng = np.random.default_rng(11)
    s = oracle.slots
    z1 = rng.uniform(-1, 1, s) + 1j * rng.uniform(-1, 1, s)
    z2 = rng.uniform(-1, 1, s) + 1j * rng.uniform(-1, 1, s)
    M = rng.uniform(-4, 4, (s, s))
    M[np.abs(M) < 1.0] = 0.0  # some zero entries; keep some diagonals
    M[:, :] *= (np.add.outer(np.arange(s), -np.arange(s)) % 3 != 1)  # zero whole diagonals
    res = {}
    for e, k in ((oracle, ko), (product, kp)):
        pk, sk, rk, rlk = k
        a, b = e.encrypt(z1, pk), e.encrypt(z2, pk)
        out = {}
        for op in ("add", "sub"):
            c = e.ct()
            getattr(e, op)(c, a, b)
            out[op] = c
        c = e.ct(); e.copy_ct(c, a); e.neg(c); out["neg"] = c
        c = e.ct(); e.copy_ct(c, a); e.moddown(c); out["moddown"] = c
        c = e.ct(); e.rot(c, a, 3, rk); out["rot3"] = c
        c = e.ct(); e.gemv(c, M.ravel(), a, rk); out["gemv"] = c
        c = e.ct(); e.mul(c, a, b, rlk); out["mul"] = c
        c = e.ct(); e.mul_rescale(c, a, b, rlk); out["mul_rescale"] = c
        c = e.ct(); e.mul(c, a, b, rlk); e.rescale(c); out["mul_then_rescale"] = c
        # in place (out aliases an operand): the fused path must not form d0/d1
        # from inputs it is overwriting
        c = e.ct(); e.copy_ct(c, a); e.mul_rescale(c, c, b, rlk); out["mul_rescale_inplace"] = c
        c = e.ct(); e.copy_ct(c, b); e.mul(c, a, c, rlk); out["mul_inplace"] = c
        res[e.name] = (out, sk)
    for op in res["oracle"][0]:
        same(oracle, product, res["oracle"][0][op], res["product"][0][op])
    # decoded sanity on the product side
    out, sk = res["product"]
    expect = {"add": z1 + z2, "sub": z1 - z2, "neg": -z1, "moddown": z1, "rot3": np.roll(z1, -3),
              "gemv": M @ z1, "mul": z1 * z2, "mul_rescale": z1 * z2, "mul_then_rescale": z1 * z2,
              "mul_rescale_inplace": z1 * z2, "mul_inplace": z1 * z2}
    for op, want in expect.items():
        got = product.decrypt(out[op], sk)
        assert np.abs(got - want).max() < 1e-6 * max(1.0, np.abs(want).max()), op


@pytest.mark.parametrize("name", ["bench", "bench51", "c5", "c5f", "c14", "c15", "f13", "f15"])
@pytest.mark.parametrize("npolys", [4, 24])
def test_ntt_batch_bitexact(oracle, product, name, npolys):
    """Config 2 layout (n=2^16, L=8) and the n=2^17, L=12 chain: forward, then
    inverse (the roundtrip identity).  4 polys run the one-tile-per-workgroup
    row pass; 24 the multi-poly row pass with staged twiddles (3 polys per
    quarter stream, the next one prefetched)."""
    import torch
    init_both(oracle, product, name)
    n, L = product.n, product.L
    host = np.zeros(npolys * L * n, dtype=np.uint64)
    oracle.lib.poly_fill_uniform(host.ctypes.data, npolys, L, 99)
    orig = host.copy()
    dev = torch.empty(npolys * L * n, dtype=torch.int64, device="cuda")
    torch.cuda.synchronize()
    product.lib.poly_fill_uniform(dev.data_ptr(), npolys, L, 99)
    product.sync()
    assert np.array_equal(dev.cpu().numpy().view(np.uint64), host)
    oracle.lib.poly_ntt_batch(host.ctypes.data, npolys, L)
    product.lib.poly_ntt_batch(dev.data_ptr(), npolys, L)
    product.sync()
    assert np.array_equal(dev.cpu().numpy().view(np.uint64), host)
    oracle.lib.poly_intt_batch(host.ctypes.data, npolys, L)
    product.lib.poly_intt_batch(dev.data_ptr(), npolys, L)
    product.sync()
    assert np.array_equal(dev.cpu().numpy().view(np.uint64), host)
    assert np.array_equal(host, orig)


@pytest.mark.parametrize("name,npolys", [("bench51", 1024), ("bench", 113)])
def test_ntt_batch_full_shape(oracle, product, name, npolys):
    """Config 2 at its full shape (1024 polys x 8 limbs at
    N=2^16, the bench's prime set) and 113 polys on the 60-bit set: ntt_batch
    runs the batch in groups of 224 MiB (api.cpp ntt_batch: 56 polys of 8
    limbs at this shape), so these cover every group offset, the row pass's
    member split at a full group and a one-poly last group (113 = 56 + 56 +
    1), which the inverse batch (GPQHE_NTT_REV) visits first.  Forward and
    inverse are each compared residue by residue with the oracle, not only
    the roundtrip."""
    import torch
    init_both(oracle, product, name)
    n, L = product.n, product.L
    host = np.zeros(npolys * L * n, dtype=np.uint64)
    oracle.lib.poly_fill_uniform(host.ctypes.data, npolys, L, 0x48454354520001)
    dev = torch.empty(npolys * L * n, dtype=torch.int64, device="cuda")
    torch.cuda.synchronize()
    product.lib.poly_fill_uniform(dev.data_ptr(), npolys, L, 0x48454354520001)
    product.sync()
    assert np.array_equal(dev.cpu().numpy().view(np.uint64), host)
    for fwd in (True, False):
        fn = "poly_ntt_batch" if fwd else "poly_intt_batch"
        getattr(oracle.lib, fn)(host.ctypes.data, npolys, L)
        getattr(product.lib, fn)(dev.data_ptr(), npolys, L)
        product.sync()
        got = dev.cpu().numpy().view(np.uint64)
        bad = np.flatnonzero(got != host)
        assert bad.size == 0, f"{fn}: {bad.size} residues differ, first at poly {bad[0] // (L * n)}"
        del got
    del host, dev


def mul_batch_both(oracle, product, name, cnt, lvl=None, seeds=(1, 2)):
    """he_mul_rescale_batch of `cnt` random-residue pairs at level `lvl` on
    both engines (same keys, same inputs); returns (oracle, product) outputs."""
    import ctypes
    import torch
    init_both(oracle, product, name)
    n = product.n
    lvl = lvl or product.L
    _, _, _, rlk_o = keys(oracle, rot=False)
    _, _, _, rlk_p = keys(product, rot=False)
    same(oracle, product, rlk_o, rlk_p)
    words = max(cnt, 1) * 2 * lvl * n
    a = np.zeros(words, dtype=np.uint64)
    b = np.zeros(words, dtype=np.uint64)
    oracle.lib.poly_fill_uniform(a.ctypes.data, 2 * max(cnt, 1), lvl, seeds[0])
    oracle.lib.poly_fill_uniform(b.ctypes.data, 2 * max(cnt, 1), lvl, seeds[1])
    out_o = np.full(max(cnt, 1) * 2 * (lvl - 1) * n, 7, dtype=np.uint64)
    oracle.lib.he_mul_rescale_batch(out_o.ctypes.data, a.ctypes.data, b.ctypes.data, cnt, lvl, ctypes.byref(rlk_o))
    da = torch.from_numpy(a.view(np.int64)).cuda()
    db = torch.from_numpy(b.view(np.int64)).cuda()
    del a, b
    dout = torch.full((out_o.size,), 7, dtype=torch.int64, device="cuda")
    torch.cuda.synchronize()
    product.lib.he_mul_rescale_batch(dout.data_ptr(), da.data_ptr(), db.data_ptr(), cnt, lvl, ctypes.byref(rlk_p))
    product.sync()
    got = dout.cpu().numpy().view(np.uint64)
    del da, db, dout
    return out_o, got


@pytest.mark.parametrize("name", ["bench", "bench_d2", "bench51", "c5", "c5f", "c17", "c14", "c15", "f13", "f15",
                                  "a5", "m60"])
def test_mul_rescale_batch_bitexact(oracle, product, name):
    """Config 3 op at n=2^16, L=8 (dnum=8/K=1 through the streaming inner
    product, the bench's dnum=2/K=4 with 60-bit and with < 2^51 primes), the
    config 5 op at n=2^17, L=12, and the other fused tilings, on 3
    random-residue pairs (one pair per quarter stream of the split key switch)."""
    want, got = mul_batch_both(oracle, product, name, 3)
    assert np.array_equal(got, want), f"{np.count_nonzero(got != want)} residues differ"


@pytest.mark.parametrize("name,cnt,chunk", [("bench51", 17, None), ("bench51", 24, None), ("bench_d2", 17, None),
                                            ("bench51", 17, 5), ("bench51", 256, None), ("bench_d2", 256, None),
                                            ("c5", 17, None), ("c5", 64, None), ("c5f", 17, None), ("c5f", 64, None),
                                            ("c15", 17, None), ("m60", 17, None)])
def test_mul_rescale_batch_bench_shape(oracle, product, name, cnt, chunk, monkeypatch):
    """The headline shape (bench.py): n=2^16, L=8,
    dnum=2, K=4 on 17 and 24 pairs (the split key switch's pair ranges of
    5-8 pairs per workgroup, two or three per quarter stream: the next pair's
    prefetch, the key tile shared by the quarters and reused across pairs,
    the accumulator restart), 17 pairs in chunks of 5/5/5/2 (the multi-chunk
    loop, a short last chunk) and the bench's own 256 pairs (one chunk of the
    8 GiB workspace, run as two 128-pair sub-chunks on two streams of that
    one chunk, about 3 pairs per quarter), every output residue compared with the oracle.  Also 17
    pairs of config 5 (n=2^17, L=12,
    the three-digit split key switch), config 5's own bench shape (64 pairs per
    GPU, bench.py's c5 leg: its pair ranges and member split), both on the
    60-bit q0/P set and on the headline's all-FP64 prime sizes (c5f), and 17 of c15
    (integer moduli: two pair streams per workgroup)."""
    if chunk:
        monkeypatch.setenv("GPQHE_CHUNK", str(chunk))
    want, got = mul_batch_both(oracle, product, name, cnt, seeds=(21, 22))
    assert np.array_equal(got, want), f"{np.count_nonzero(got != want)} residues differ"


@pytest.mark.parametrize("streams", [1, 2])
def test_mul_rescale_batch_streams(oracle, product, streams):
    """The batch as one chunk on the engine stream (gpqhe_set_streams(1)) and
    as two sub-chunks on two streams, the second started after the first's
    d2_rows (the default): identical residues either way, odd split 12 + 13."""
    product.lib.gpqhe_set_streams(streams)
    try:
        want, got = mul_batch_both(oracle, product, "bench51", 25, seeds=(31, 32))
    finally:
        product.lib.gpqhe_set_streams(2)
    assert np.array_equal(got, want), f"{np.count_nonzero(got != want)} residues differ"


@pytest.mark.parametrize("name", ["bench_d2", "bench51"])
def test_batch_real_encryptions_decode(product, name):
    """a 4-ciphertext subset of real encryptions of
    uniform reals in [-1, 1] through he_mul_rescale_batch decodes to the
    slot-wise products, on the conventional 60-bit q0/P set and on the
    bench's < 2^51 set (q0 51 bits at Delta = 2^50)."""
    import ctypes
    import torch
    kind, kw = PARAMS[name]
    product.init_params(**kw)
    product.set_seed(9)
    pk, sk, _, rlk = keys(product, rot=False)
    n, L, s, cnt = product.n, product.L, product.slots, 4
    rng = np.random.default_rng(12)
    za = rng.uniform(-1, 1, (cnt, s)) + 1j * rng.uniform(-1, 1, (cnt, s))
    zb = rng.uniform(-1, 1, (cnt, s)) + 1j * rng.uniform(-1, 1, (cnt, s))
    ha = np.concatenate([product.export(product.encrypt(z, pk)).ravel() for z in za])
    hb = np.concatenate([product.export(product.encrypt(z, pk)).ravel() for z in zb])
    da = torch.from_numpy(ha.view(np.int64)).cuda()
    db = torch.from_numpy(hb.view(np.int64)).cuda()
    dout = torch.zeros(cnt * 2 * (L - 1) * n, dtype=torch.int64, device="cuda")
    torch.cuda.synchronize()
    product.lib.he_mul_rescale_batch(dout.data_ptr(), da.data_ptr(), db.data_ptr(), cnt, L, ctypes.byref(rlk))
    product.sync()
    out = dout.cpu().numpy().view(np.uint64).reshape(cnt, -1)
    delta = product.info.delta
    for i in range(cnt):
        ct = product.ct()
        product.import_(ct, out[i], L - 1, scale=delta * delta / product.primes[L - 1])
        got = product.decrypt(ct, sk)
        assert np.abs(got - za[i] * zb[i]).max() < 1e-6
        product.free(ct)


@pytest.mark.parametrize("frac,ok", [(0.8, True), (1.3, False)])
def test_batch_level0_headroom(product, frac, ok):
    """The bench's < 2^51 set (q0 51 bits at Delta = 2^50) keeps about one bit
    of integer headroom once a product lands on q0 alone.  A constant real
    slot vector (m(X) = c * Delta, the worst case for the coefficient bound)
    is encrypted on two limbs, multiplied and rescaled by he_mul_rescale_batch
    down to q0: a product below q0 / (2 * scale) decodes exactly, one above
    it wraps modulo q0 -- the capacity is stated, not hidden."""
    import ctypes
    import torch
    kind, kw = PARAMS["bench51"]
    product.init_params(**kw)
    product.set_seed(3)
    pk, sk, _, rlk = keys(product, rot=False)
    n, s, lvl = product.n, product.slots, 2
    delta = product.info.delta
    scale = delta * delta / product.primes[lvl - 1]
    cap = product.primes[0] / 2 / scale
    c = np.sqrt(frac * cap)
    z = np.full(s, c, dtype=np.complex128)
    h = product.export(product.encrypt(z, pk, nlimbs=lvl)).ravel()
    da = torch.from_numpy(h.view(np.int64)).cuda()
    dout = torch.zeros(2 * (lvl - 1) * n, dtype=torch.int64, device="cuda")
    torch.cuda.synchronize()
    product.lib.he_mul_rescale_batch(dout.data_ptr(), da.data_ptr(), da.data_ptr(), 1, lvl, ctypes.byref(rlk))
    product.sync()
    ct = product.ct()
    product.import_(ct, dout.cpu().numpy().view(np.uint64), lvl - 1, scale=scale)
    err = np.abs(product.decrypt(ct, sk) - c * c).max()
    product.free(ct)
    if ok:
        assert err < 1e-6, err
    else:
        assert abs(err - product.primes[0] / scale) < 1e-3, (err, product.primes[0] / scale)


@pytest.mark.parametrize("name,lvl,cnt", [("bench51", 6, 2), ("bench_d2", 3, 2), ("bench51", 8, 1),
                                          ("bench51", 8, 0)])
def test_mul_rescale_batch_levels(oracle, product, name, lvl, cnt):
    """The fused batch op below the top level (lvl 6: digits {0..3} {4,5},
    a partial digit; lvl 3: one partial digit), a batch of one pair and an
    empty batch (a no-op that must not touch the output)."""
    want, got = mul_batch_both(oracle, product, name, cnt, lvl=lvl, seeds=(5, 6))
    assert np.array_equal(got, want), f"{np.count_nonzero(got != want)} residues differ"
    if cnt == 0:
        assert np.all(got == 7)


def test_gemv_zero_matrix(oracle, product):
    """he_gemv with an all-zero matrix (no diagonal is launched): the output is
    an encryption of zero, bit-exact with the oracle."""
    init_both(oracle, product, "ref")
    res = {}
    z = np.linspace(-1, 1, oracle.slots) + 0j
    M = np.zeros((oracle.slots, oracle.slots))
    for e in (oracle, product):
        pk, sk, rk, _ = keys(e)
        x = e.encrypt(z, pk)
        y = e.ct()
        e.gemv(y, M.ravel(), x, rk)
        res[e.name] = (e, y, sk)
    same(oracle, product, res["oracle"][1], res["product"][1])
    e, y, sk = res["product"]
    assert np.abs(e.decrypt(y, sk)).max() < 1e-6


@pytest.mark.parametrize("name", ["ref", "c1", "hyb"])
def test_gemv_queue(oracle, product, name):
    """Queued he_gemv calls (api.cpp:flush_gemvs): two independent gemvs run as
    one batch (one ModUp over both inputs, one inner-product launch, one
    ModDown with two outputs: the fused small-N kernels at n=4096, the
    down_combine two-output split at n=2^13); a third that reads the second's
    output and an all-zero matrix queued beside a non-zero one.  Every output
    bit-exact with the oracle's sequential calls."""
    init_both(oracle, product, name)
    rng = np.random.default_rng(17)
    s = oracle.slots
    z1 = rng.uniform(-1, 1, s) + 0j
    z2 = rng.uniform(-1, 1, s) + 0j
    M1, M2, M3 = (rng.uniform(-2, 2, (s, s)) for _ in range(3))
    Z = np.zeros((s, s))
    res = {}
    for e in (oracle, product):
        pk, sk, rk, _ = keys(e)
        a, b = e.encrypt(z1, pk), e.encrypt(z2, pk)
        y1, y2, y3, y4, y5 = (e.ct() for _ in range(5))
        e.gemv(y1, M1.ravel(), a, rk)
        e.gemv(y2, M2.ravel(), b, rk)  # independent: batched with y1
        chain = e.L >= 3  # y2 is one level down; HECTR's own L = 2 has no room for a second gemv
        e.gemv(y3, M3.ravel(), y2 if chain else a, rk)  # reads y2: runs after the batch
        e.gemv(y4, Z.ravel(), a, rk)  # all-zero matrix queued beside y5
        e.gemv(y5, M1.ravel(), b, rk)
        res[e.name] = ([y1, y2, y3, y4, y5], sk)
    for o, p in zip(res["oracle"][0], res["product"][0]):
        same(oracle, product, o, p)
    ys, sk = res["product"]
    want = [M1 @ z1, M2 @ z2, M3 @ (M2 @ z2) if product.L >= 3 else M3 @ z1, 0 * z1, M1 @ z2]
    for y, w in zip(ys, want):
        assert np.abs(product.decrypt(y, sk) - w).max() < 1e-5 * max(1.0, np.abs(w).max())



@pytest.mark.parametrize("name,slots", [("c1", 2048), ("c1", 4096), ("bench51", 32768), ("bench51", 4096)])
def test_gpu_encode_bitexact(oracle, product, name, slots):
    """he_ecd with the special FFT on the GPU (slot counts
    >= GPQHE_GPU_ECD_MIN = 2048): the LDS-only transform (2048 slots) and the
    global + LDS stages (4096 and the full n/2 = 32768 slots at n=2^16) give
    the host/oracle encoding bit for bit, and it decrypts to the input."""
    init_both(oracle, product, name)
    rng = np.random.default_rng(slots)
    z = rng.uniform(-1, 1, slots) + 1j * rng.uniform(-1, 1, slots)
    delta = product.info.delta
    res = {}
    for e in (oracle, product):
        pt = e.pt()
        e.ecd_ex(pt, z, slots, delta, e.L)
        res[e.name] = e.export(pt)
        e.free(pt)
    assert np.array_equal(res["oracle"], res["product"]), \
        f"{np.count_nonzero(res['oracle'] != res['product'])} residues differ"
    pk, sk, _, _ = keys(product, rot=False)
    pt, ct, dec = product.pt(), product.ct(), product.pt()
    product.ecd_ex(pt, z, slots, delta, product.L)
    product.enc_pk(ct, pt, pk)
    product.dec(dec, ct, sk)
    got = product.dcd(dec, slots)
    assert np.abs(got - z).max() < 1e-6
    for o in (pt, ct, dec):
        product.free(o)


@pytest.mark.parametrize("name,slots,nl", [("ref", 16, 2), ("ref", 2048, 1), ("c1", 64, 3), ("c1", 4096, 4),
                                           ("bench51", 32768, 8), ("c5", 8192, 12)])
def test_gpu_decode_bitexact(oracle, product, name, slots, nl):
    """he_dcd on the GPU (kernels.hip k_decode: centred CRT lift + special
    forward FFT) against the oracle's host decode, bit for bit.  Uniform random
    residues decode to full-width values of both signs (|x| up to Q/2, every
    word of the multi-word lift); both the NTT-form input (inverse transform
    first) and a coefficient-form one (GPQHE_F_COEFF).  Slot counts cover one
    LDS chunk (16..2048) and the global stages above 2048; nl = 1 (the
    single-limb shortcut) up to 12 limbs."""
    init_both(oracle, product, name)
    n = product.n
    rng = np.random.default_rng(slots + nl)
    res = np.stack([rng.integers(0, q, n, dtype=np.uint64) for q in product.primes[:nl]])
    # small centred values on a second plaintext: the decrypt-range branch
    small = rng.integers(-2 ** 40, 2 ** 40, n)
    res_small = np.stack([(small % q).astype(np.uint64) for q in product.primes[:nl]])
    scale = 2.0 ** 40
    for arr in (res, res_small):
        for flags in (0, 1):
            got = {}
            for e in (oracle, product):
                pt = e.pt()
                e.import_(pt, arr, nl, scale, flags)
                got[e.name] = e.dcd(pt, slots)
                e.free(pt)
            o, p = got["oracle"], got["product"]
            assert np.array_equal(o.view(np.uint64), p.view(np.uint64)), \
                f"{np.count_nonzero(o != p)} of {slots} decoded slots differ (flags={flags})"


@pytest.mark.parametrize("name", ["ref", "c1"])
def test_ew_queue_sequences(oracle, product, name):
    """The queued elementwise calls at n <= 2^12 (api.cpp g_pew: he_add /
    he_sub / he_neg / he_copy_ct / he_dec as one ew_prog_kernel launch) keep
    call order: aliasing outputs, a level drop (he_moddown) between queued
    ops, a freed object whose block is handed out again while queued ops
    still name it (next user queued, and next user an unqueued he_mul), and a
    decryption queued behind them -- bit-exact vs the oracle's sequential
    calls.  At n = 2^13 (c1) the same calls run unqueued."""
    init_both(oracle, product, name)
    rng = np.random.default_rng(11)
    z1 = rng.uniform(-1, 1, oracle.slots) + 0j
    z2 = rng.uniform(-1, 1, oracle.slots) + 0j
    out = {}
    for e in (oracle, product):
        pk, sk, _, rlk = keys(e, rot=False)
        a, b = e.encrypt(z1, pk), e.encrypt(z2, pk)
        c = e.ct()
        e.sub(c, a, b)
        e.add(c, c, a)          # out aliases an input
        e.neg(c)
        d = e.ct()
        e.copy_ct(d, c)
        e.moddown(d)            # level drop between queued ops
        g = e.ct()
        e.add(g, d, a)          # mixed levels: min
        e.free(c)               # c's block is free while ops naming it are queued
        f = e.ct()
        e.sub(f, a, b)          # queued user of the reused block
        e.free(f)
        h = e.ct()
        e.mul(h, a, b, rlk)     # unqueued user of a reused block
        pt = e.pt()
        e.dec(pt, g, sk)
        out[e.name] = [e.export(x) for x in (d, g, h, pt)] + [e.dcd(pt)]
    for i, (x, y) in enumerate(zip(out["oracle"], out["product"])):
        assert np.array_equal(x, y), f"object {i} differs"
    assert np.abs(out["product"][4] - (-(z1 - z2 + z1) + z1)).max() < 1e-6


@pytest.mark.parametrize("slot_set", [(16,) * 5, (16, 2, 512, 1), (1024,) * 5],
                         ids=["kernel_args", "pinned_map", "upload"])
def test_queued_encodes_mixed_slots(oracle, product, slot_set):
    """Queued he_ecd_ex at n = 4096 pass only the coefficients on the widest
    stride all queued encodes share (api.cpp flush_pending, clog), in the
    kernel arguments (HECTR's 5 x 16 slots), read from pinned host memory
    (16, 2, 512 and 1 slots: 4 x 1024 values) or uploaded (5 x 1024 slots),
    then encryptions of them, bit-exact vs the oracle."""
    init_both(oracle, product, "ref")
    rng = np.random.default_rng(4)
    zs = [rng.uniform(-1, 1, s) + 1j * rng.uniform(-1, 1, s) for s in slot_set]
    out = {}
    for e in (oracle, product):
        pk, sk, _, _ = keys(e, rot=False)
        pts, cts = [], []
        for z in zs:
            pt = e.pt()
            e.ecd_ex(pt, z, len(z), e.info.delta, e.L)
            pts.append(pt)
        for pt in pts:
            ct = e.ct()
            e.enc_pk(ct, pt, pk)
            cts.append(ct)
        out[e.name] = [e.export(x) for x in pts + cts]
    for i, (x, y) in enumerate(zip(out["oracle"], out["product"])):
        assert np.array_equal(x, y), f"object {i} differs"


@pytest.mark.parametrize("slot_set", [(16,) * 5, (16, 2, 512, 1), (1024,) * 5],
                         ids=["kernel_args", "pinned_map", "upload"])
def test_queued_encryptions_freed_plaintexts(oracle, product, slot_set):
    """HECTR's step (reference src/ctr.c:466-480): encodes and encryptions
    queued, then the plaintexts freed before anything ran.  A freed encode is
    dropped and its encryption adds the plaintext's coefficients to e0 before
    the transform (api.cpp drop_dead_encode, kernels.hip EncCoef); one
    plaintext stays live, and a freed block is encoded into and encrypted
    again while the dropped encode is still queued -- bit-exact vs the
    oracle's sequential calls, and the decryptions within the CKKS tolerance."""
    init_both(oracle, product, "ref")
    rng = np.random.default_rng(8)
    zs = [rng.uniform(-1, 1, s) + 1j * rng.uniform(-1, 1, s) for s in slot_set]
    out = {}
    for e in (oracle, product):
        pk, sk, _, _ = keys(e, rot=False)
        pts, cts = [], []
        for z in zs:
            pt = e.pt()
            e.ecd_ex(pt, z, len(z), e.info.delta, e.L)
            pts.append(pt)
        for pt in pts:
            ct = e.ct()
            e.enc_pk(ct, pt, pk)
            cts.append(ct)
        for i, pt in enumerate(pts):
            if i != 1:
                e.free(pt)
        pt2 = e.pt()  # may take a freed plaintext's block
        e.ecd_ex(pt2, zs[0], len(zs[0]), e.info.delta, e.L)
        ct2 = e.ct()
        e.enc_pk(ct2, pt2, pk)
        out[e.name] = [e.export(x) for x in cts + [pts[1], pt2, ct2]]
        if e is product:
            for z, ct in zip(zs, cts):
                assert np.abs(e.decrypt(ct, sk, len(z)) - z).max() < 1e-6
    for i, (x, y) in enumerate(zip(out["oracle"], out["product"])):
        assert np.array_equal(x, y), f"object {i} differs"


def test_speculative_encryption_noise(oracle, product):
    """The small-N step's speculative noise (api.cpp SpecNoise): after each
    he_dcd the noise of the next step's encryptions is sampled ahead, and a
    flush whose encryptions take exactly those streams only runs the combine,
    evaluating the plaintexts from their coefficients (k_enc_combine_m).
    Steps of 5 encryptions (HECTR's), then 3 (a prefix of the speculated
    streams), 6 (more than speculated), one of a live plaintext, an
    encryption at a lower level, and a reseed between steps -- every
    ciphertext bit-exact vs the oracle's sequential calls
    (tests/small_n_steps.py)."""
    from tests.small_n_steps import mismatches, speculative_noise
    assert mismatches(speculative_noise(oracle), speculative_noise(product)) == []


def test_gemv_of_queued_differences(oracle, product):
    """HECTR's regulator step (src/hempc.c:253-270) repeated: he_sub x2 of
    fresh encryptions, he_gemv of each difference (api.cpp ew_lazy_sub: from
    the second step on, the subs stay queued and gemv_inner_kernel forms the
    differences from their operands), then he_add / he_neg and the decode.
    Variants per step: the differences freed unread (their queued subs are
    dropped), read back after the gemvs (the subs must still run), an operand
    of a sub overwritten after the gemvs (the gemv must see the old value),
    GPQHE-style non-speculated steps (a different number of encryptions),
    an in-place he_gemv(x, M, x) and a gemv whose output is an operand of the
    queued sub (the lazy form must not run the gemv ahead of those subs:
    ADVICE r3) -- every exported object and decoded value bit-exact vs the
    oracle (tests/small_n_steps.py)."""
    from tests.small_n_steps import mismatches, queued_differences
    assert mismatches(queued_differences(oracle), queued_differences(product)) == []


def test_speculative_gemvs(oracle, product):
    """The speculated gemv of the small-N step (api.cpp SpecGemv): HECTR's own
    call order, taken from the third step on, and the steps where it must not
    be taken (a changed matrix, swapped operands, an encryption overwritten
    before its he_sub, the gemvs in the other order, keys regenerated in place,
    one gemv only) -- bit-exact vs the oracle, and the product served some
    he_gemv calls from the speculation."""
    from tests.small_n_steps import mismatches, speculative_gemvs
    want = speculative_gemvs(oracle)
    got = speculative_gemvs(product)
    taken = product.lib.gpqhe_spec_gemv_taken()
    assert mismatches(want, got) == []
    assert taken >= 10, taken


def test_speculative_decode(oracle, product, monkeypatch):
    """The replayed tail of the small-N step (api.cpp SpecDcd: the last step's
    elementwise program and decode on this step's speculated gemvs): runs of
    HECTR's step in its own call order, broken by steps whose program or
    operands differ (a changed matrix, an encryption overwritten before its
    he_sub, the gemvs in the other order, one gemv, a speculated result's
    block handed to a gemv that is not speculated), where the replay must not
    be taken -- every decoded value and object bit-exact vs the oracle, and the
    product served decodes from the replay."""
    from tests.small_n_steps import mismatches, speculative_gemvs
    plan = ["same"] * 7 + ["newM", "same", "same", "same", "clobber"] + ["same"] * 4 + ["order"] + ["same"] * 4 + \
        ["one"] + ["same"] * 4 + ["realias"] + ["same"] * 4
    # (a Python caller outruns the device: keep the replay on, which the
    # library otherwise stops after two late steps)
    monkeypatch.setenv("GPQHE_SPEC_DCD", "2")
    want = speculative_gemvs(oracle, plan=plan)
    got = speculative_gemvs(product, plan=plan)
    dcd = product.lib.gpqhe_spec_dcd_taken()
    assert mismatches(want, got) == []
    assert dcd >= 5, dcd


def test_rekey_between_speculative_steps(oracle, product):
    """The speculative ModUp is keyed on the public key's block (api.cpp
    SpecModup / C1Prov): re-keying between steps -- the key freed and a new
    he_keypair that may take its block, then two keys alternating step by
    step -- must never reuse digits made with another key's values; bit-exact
    vs the oracle."""
    from tests.small_n_steps import mismatches, rekeyed_steps
    assert mismatches(rekeyed_steps(oracle), rekeyed_steps(product)) == []


@pytest.mark.parametrize("switch", ["GPQHE_SPEC", "GPQHE_SPEC_ATTACH", "GPQHE_SPEC_EARLY", "GPQHE_DEFER",
                                    "GPQHE_DEFER_SUB", "GPQHE_DEFER_GEMV", "GPQHE_SPEC_ATTACH_TAKE",
                                    "GPQHE_SPEC_GEMV", "GPQHE_SPEC_MODUP_SPLIT", "GPQHE_SPEC_DCD"])
def test_small_n_switch_off_paths(switch):
    """Each small-N switch is read once per process (api.cpp static const), so
    its off path runs in a child process (one at a time, nothing else on the
    GPU meanwhile): the three step sequences of tests/small_n_steps.py with
    the switch at 0, bit-exact vs the oracle."""
    import json
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, **{switch: "0"})
    r = subprocess.run([sys.executable, os.path.join(root, "tests", "switch_worker.py")], env=env, cwd=root,
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    res = json.loads(r.stdout.strip().splitlines()[-1])
    assert res == {k: [] for k in res} and len(res) == 4, res


@pytest.mark.parametrize("name", ["ref", "c1"])
def test_plaintext_ops_rot0_and_queue_overflow(oracle, product, name):
    """he_add_pt (out != a: a queued copy the add then reads; and in place),
    he_mul_pt, he_rot by 0 (a queued copy at n <= 2^12), and a chain of 20
    he_add calls (40 queued entries: the elementwise queue runs whenever 16
    fill up) -- bit-exact vs the oracle."""
    init_both(oracle, product, name)
    rng = np.random.default_rng(21)
    s = oracle.slots
    z1 = rng.uniform(-1, 1, s) + 0j
    z2 = rng.uniform(-1, 1, s) + 0j
    res = {}
    for e in (oracle, product):
        pk, sk, rk, _ = keys(e)
        a = e.encrypt(z1, pk)
        pt = e.pt()
        e.ecd(pt, z2)
        out = {}
        c = e.ct(); e.add_pt(c, a, pt); out["add_pt"] = c
        c = e.ct(); e.copy_ct(c, a); e.add_pt(c, c, pt); out["add_pt_inplace"] = c
        c = e.ct(); e.mul_pt(c, a, pt); out["mul_pt"] = c
        c = e.ct(); e.rot(c, a, 0, rk); out["rot0"] = c
        c = e.ct(); e.copy_ct(c, a)
        for _ in range(20):
            e.add(c, c, a)
        out["add_chain"] = c
        res[e.name] = {k: e.export(v) for k, v in out.items()}
        if e is product:
            assert np.abs(e.decrypt(out["add_chain"], sk) - 21 * z1).max() < 1e-5
            assert np.abs(e.decrypt(out["add_pt"], sk) - (z1 + z2)).max() < 1e-6
    for k in res["oracle"]:
        assert np.array_equal(res["oracle"][k], res["product"][k]), k
