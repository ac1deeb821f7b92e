"""ctypes binding of the GPQHE C ABI (include/gpqhe.h).

One class, two engines:
  * ``Engine.product()`` loads the in-tree ``hectr_amd/lib/libgpqhe.so`` (the
    MI355X product: host C++ + gfx950 HIP kernels).  It raises if the library
    is missing -- there is no CPU fallback on the product path.
  * ``Engine.oracle()`` loads ``oracle/libgpqhe_oracle.so``, the CPU C
    restatement.  Only tests/, __graft_entry__.smoke() and bench.py's
    cpu_baseline leg use it, as the checker / CPU baseline.

The methods mirror HECTR's call sites of the GPQHE API (reference
src/ctr.c:445-618, src/hempc.c:216-274): same names, same argument order
(output first), same void/abort error behaviour.
"""
from __future__ import annotations

import ctypes as C
import os
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent.parent
PRODUCT_LIB = ROOT / "hectr_amd" / "lib" / "libgpqhe.so"
ORACLE_LIB = ROOT / "oracle" / "libgpqhe_oracle.so"

F_COEFF = 1
F_SPECIAL = 2


class HeObject(C.Structure):
    """GPQHE_OBJECT_FIELDS (include/gpqhe.h)."""

    _fields_ = [
        ("data", C.POINTER(C.c_uint64)),
        ("nlimbs", C.c_uint32),
        ("cap", C.c_uint32),
        ("npoly", C.c_uint32),
        ("galois", C.c_uint32),
        ("scale", C.c_double),
        ("flags", C.c_uint32),
        ("dnum", C.c_uint32),
        ("reserved", C.c_uint64),
    ]


class Params(C.Structure):
    _fields_ = [
        ("logn", C.c_uint32),
        ("nlimbs", C.c_uint32),
        ("nspecial", C.c_uint32),
        ("dnum", C.c_uint32),
        ("slots", C.c_uint32),
        ("q0_bits", C.c_uint32),
        ("qi_bits", C.c_uint32),
        ("p_bits", C.c_uint32),
        ("delta", C.c_double),
        ("seed", C.c_uint64),
    ]


class Info(C.Structure):
    _fields_ = [
        ("logn", C.c_uint32),
        ("n", C.c_uint32),
        ("nlimbs", C.c_uint32),
        ("nspecial", C.c_uint32),
        ("dnum", C.c_uint32),
        ("alpha", C.c_uint32),
        ("slots", C.c_uint32),
        ("reserved", C.c_uint32),
        ("delta", C.c_double),
        ("primes", C.c_uint64 * 64),
        ("psi", C.c_uint64 * 64),
    ]


class KStat(C.Structure):
    _fields_ = [("name", C.c_char * 40), ("launches", C.c_uint32), ("reserved", C.c_uint32),
                ("total_us", C.c_double), ("bytes", C.c_double)]


P = C.POINTER
OBJ = P(HeObject)
VP = C.c_void_p
U64P = P(C.c_uint64)

# name -> (restype, argtypes); every entry is exported by both libraries.
SIGNATURES = {
    "gpqhe_mpi_set_ui": (VP, [VP, C.c_ulong]),
    "gpqhe_mpi_lshift": (None, [VP, VP, C.c_uint]),
    "gpqhe_mpi_release": (None, [VP]),
    "gpqhe_mpi_get_nbits": (C.c_uint, [VP]),
    "hectx_init": (None, [C.c_uint, VP, C.c_uint, C.c_uint64]),
    "hectx_exit": (None, []),
    "hectx_init_params": (None, [P(Params)]),
    "hectx_info": (None, [P(Info)]),
    "gpqhe_set_seed": (None, [C.c_uint64]),
    "gpqhe_set_stream": (None, [VP]),
    "gpqhe_set_streams": (None, [C.c_uint]),
    "gpqhe_sync": (None, []),
    "he_alloc_pk": (None, [OBJ]), "he_free_pk": (None, [OBJ]),
    "he_alloc_sk": (None, [OBJ]), "he_free_sk": (None, [OBJ]),
    "he_alloc_evk": (None, [OBJ]), "he_free_evk": (None, [OBJ]),
    "he_alloc_ct": (None, [OBJ]), "he_free_ct": (None, [OBJ]),
    "he_alloc_pt": (None, [OBJ]), "he_free_pt": (None, [OBJ]),
    "he_keypair": (None, [OBJ, OBJ]),
    "he_genrk": (None, [OBJ, OBJ]),
    "he_genrlk": (None, [OBJ, OBJ]),
    "he_genrot": (None, [OBJ, C.c_uint, OBJ]),
    "he_ecd": (None, [OBJ, VP]),
    "he_dcd": (None, [VP, OBJ]),
    "he_ecd_ex": (None, [OBJ, VP, C.c_uint, C.c_double, C.c_uint]),
    "he_dcd_ex": (None, [VP, OBJ, C.c_uint]),
    "he_enc_pk": (None, [OBJ, OBJ, OBJ]),
    "he_enc_sk": (None, [OBJ, OBJ, OBJ]),
    "he_dec": (None, [OBJ, OBJ, OBJ]),
    "he_add": (None, [OBJ, OBJ, OBJ]),
    "he_sub": (None, [OBJ, OBJ, OBJ]),
    "he_neg": (None, [OBJ]),
    "he_copy_ct": (None, [OBJ, OBJ]),
    "he_moddown": (None, [OBJ]),
    "he_gemv": (None, [OBJ, VP, OBJ, OBJ]),
    "he_rot": (None, [OBJ, OBJ, C.c_uint, OBJ]),
    "he_mul": (None, [OBJ, OBJ, OBJ, OBJ]),
    "he_rescale": (None, [OBJ]),
    "he_mul_rescale": (None, [OBJ, OBJ, OBJ, OBJ]),
    "he_mul_pt": (None, [OBJ, OBJ, OBJ]),
    "he_add_pt": (None, [OBJ, OBJ, OBJ]),
    "he_mul_rescale_batch": (None, [VP, VP, VP, C.c_size_t, C.c_uint, OBJ]),
    "he_gemv_batch": (None, [VP, VP, VP, C.c_size_t, C.c_uint, OBJ]),
    "he_rot_batch": (None, [VP, VP, C.c_size_t, C.c_uint, C.c_uint, OBJ]),
    "poly_ntt_batch": (None, [VP, C.c_size_t, C.c_uint]),
    "poly_intt_batch": (None, [VP, C.c_size_t, C.c_uint]),
    "poly_fill_uniform": (None, [VP, C.c_size_t, C.c_uint, C.c_uint64]),
    "he_export": (C.c_size_t, [VP, U64P]),
    "he_import": (None, [VP, U64P, C.c_uint, C.c_double, C.c_uint32]),
    "he_evk_meta": (None, [OBJ, P(C.c_uint32), P(C.c_uint32)]),
    "gpqhe_prof_enable": (None, [C.c_int]),
    "gpqhe_prof_collect": (C.c_uint, [P(KStat), C.c_uint]),
    "gpqhe_spec_gemv_taken": (C.c_uint, []),
    "gpqhe_spec_dcd_taken": (C.c_uint, []),
}

#: [ext] symbols added in round 6: a library named by GPQHE_LIB (an A/B
#: baseline built from an older commit) may lack them
NEWER = {"gpqhe_spec_gemv_taken", "gpqhe_spec_dcd_taken"}

#: symbols declared in include/gpqhe.h (checked by tests/test_abi.py)
EXPORTED = sorted(SIGNATURES)


def _cplx(z) -> np.ndarray:
    return np.ascontiguousarray(np.asarray(z, dtype=np.complex128))


class Engine:
    """One loaded implementation of the GPQHE ABI."""

    def __init__(self, path: Path, name: str):
        if not Path(path).exists():
            raise FileNotFoundError(
                f"{name} library {path} is missing; run __graft_entry__.build()")
        self.path = Path(path)
        self.name = name
        self.lib = C.CDLL(str(path), mode=C.RTLD_LOCAL)
        for sym, (res, args) in SIGNATURES.items():
            if sym in NEWER and os.environ.get("GPQHE_LIB") and not hasattr(self.lib, sym):
                continue  # an older library under GPQHE_LIB (same-box A/B baselines)
            f = getattr(self.lib, sym)
            f.restype = res
            f.argtypes = args
        self.info = None

    @classmethod
    def product(cls) -> "Engine":
        return cls(Path(os.environ.get("GPQHE_LIB", PRODUCT_LIB)), "product")

    @classmethod
    def oracle(cls) -> "Engine":
        return cls(ORACLE_LIB, "oracle")

    # ---------------------------------------------------------------- ctx
    def init(self, logn: int, logq: int, slots: int, log_delta: int):
        """hectx_init(logn, q = 2^logq, slots, Delta = 2^log_delta)."""
        q = self.lib.gpqhe_mpi_set_ui(None, 1)
        self.lib.gpqhe_mpi_lshift(q, q, logq)
        self.lib.hectx_init(logn, q, slots, 1 << log_delta)
        self.lib.gpqhe_mpi_release(q)
        return self._load_info()

    def init_params(self, logn, nlimbs, slots=None, dnum=None, nspecial=1, q0_bits=60,
                    qi_bits=50, p_bits=60, delta=None, seed=1):
        p = Params(logn=logn, nlimbs=nlimbs, nspecial=nspecial, dnum=dnum or nlimbs,
                   slots=slots or (1 << (logn - 1)), q0_bits=q0_bits, qi_bits=qi_bits,
                   p_bits=p_bits, delta=float(delta or 2.0 ** qi_bits), seed=seed)
        self.lib.hectx_init_params(C.byref(p))
        return self._load_info()

    def _load_info(self):
        info = Info()
        self.lib.hectx_info(C.byref(info))
        self.info = info
        self.n = info.n
        self.L = info.nlimbs
        self.K = info.nspecial
        self.slots = info.slots
        self.primes = [info.primes[i] for i in range(info.nlimbs + info.nspecial)]
        return info

    def exit(self):
        self.lib.hectx_exit()

    def set_seed(self, seed: int):
        self.lib.gpqhe_set_seed(seed)

    def sync(self):
        self.lib.gpqhe_sync()

    def prof_enable(self, on=True):
        self.lib.gpqhe_prof_enable(1 if on else 0)

    def prof_collect(self):
        """{kernel: (launches, total_us, algorithmic bytes)}; resets the counters."""
        buf = (KStat * 64)()
        k = self.lib.gpqhe_prof_collect(buf, 64)
        return {buf[i].name.decode(): (buf[i].launches, buf[i].total_us, buf[i].bytes) for i in range(k)}

    # ------------------------------------------------------------ objects
    def _new(self, kind: str) -> HeObject:
        o = HeObject()
        getattr(self.lib, "he_alloc_" + kind)(C.byref(o))
        o._kind = kind
        return o

    def ct(self):
        return self._new("ct")

    def pt(self):
        return self._new("pt")

    def pk(self):
        return self._new("pk")

    def sk(self):
        return self._new("sk")

    def evk(self):
        return self._new("evk")

    def evks(self, count):
        arr = (HeObject * count)()
        for i in range(count):
            self.lib.he_alloc_evk(C.byref(arr[i]))
        return arr

    def free(self, o, kind=None):
        getattr(self.lib, "he_free_" + (kind or o._kind))(C.byref(o))

    def free_evks(self, arr):
        for i in range(len(arr)):
            self.lib.he_free_evk(C.byref(arr[i]))

    # --------------------------------------------------------------- API
    def keypair(self, pk, sk):
        self.lib.he_keypair(C.byref(pk), C.byref(sk))

    def genrk(self, rk, sk):
        self.lib.he_genrk(rk, C.byref(sk))

    def genrlk(self, rlk, sk):
        self.lib.he_genrlk(C.byref(rlk), C.byref(sk))

    def ecd(self, pt, z):
        z = _cplx(z)
        assert z.size >= self.slots
        self.lib.he_ecd(C.byref(pt), z.ctypes.data)

    def ecd_ex(self, pt, z, slots, scale, nlimbs):
        z = _cplx(z)
        self.lib.he_ecd_ex(C.byref(pt), z.ctypes.data, slots, scale, nlimbs)

    def dcd(self, pt, slots=None):
        s = slots or self.slots
        z = np.zeros(s, dtype=np.complex128)
        self.lib.he_dcd_ex(z.ctypes.data, C.byref(pt), s)
        return z

    def enc_pk(self, ct, pt, pk):
        self.lib.he_enc_pk(C.byref(ct), C.byref(pt), C.byref(pk))

    def enc_sk(self, ct, pt, sk):
        self.lib.he_enc_sk(C.byref(ct), C.byref(pt), C.byref(sk))

    def dec(self, pt, ct, sk):
        self.lib.he_dec(C.byref(pt), C.byref(ct), C.byref(sk))

    def add(self, out, a, b):
        self.lib.he_add(C.byref(out), C.byref(a), C.byref(b))

    def sub(self, out, a, b):
        self.lib.he_sub(C.byref(out), C.byref(a), C.byref(b))

    def neg(self, ct):
        self.lib.he_neg(C.byref(ct))

    def copy_ct(self, dst, src):
        self.lib.he_copy_ct(C.byref(dst), C.byref(src))

    def moddown(self, ct):
        self.lib.he_moddown(C.byref(ct))

    def gemv(self, y, M, x, rk):
        M = _cplx(M)
        self.lib.he_gemv(C.byref(y), M.ctypes.data, C.byref(x), rk)

    def rot(self, out, x, r, rk):
        self.lib.he_rot(C.byref(out), C.byref(x), r, rk)

    def mul(self, out, a, b, rlk):
        self.lib.he_mul(C.byref(out), C.byref(a), C.byref(b), C.byref(rlk))

    def mul_rescale(self, out, a, b, rlk):
        self.lib.he_mul_rescale(C.byref(out), C.byref(a), C.byref(b), C.byref(rlk))

    def rescale(self, ct):
        self.lib.he_rescale(C.byref(ct))

    def mul_pt(self, out, a, pt):
        self.lib.he_mul_pt(C.byref(out), C.byref(a), C.byref(pt))

    def add_pt(self, out, a, pt):
        self.lib.he_add_pt(C.byref(out), C.byref(a), C.byref(pt))

    # ------------------------------------------------------ serialization
    def export(self, o) -> np.ndarray:
        nl = o.nlimbs
        buf = np.zeros(o.npoly * nl * self.n, dtype=np.uint64)
        w = self.lib.he_export(C.byref(o), buf.ctypes.data_as(U64P))
        assert w == buf.size, (w, buf.size)
        return buf.reshape(o.npoly, nl, self.n)

    def import_(self, o, arr, nlimbs, scale=0.0, flags=0):
        arr = np.ascontiguousarray(arr, dtype=np.uint64)
        self.lib.he_import(C.byref(o), arr.ctypes.data_as(U64P), nlimbs, scale, flags)

    # ------------------------------------------------------- conveniences
    def encrypt(self, z, pk, slots=None, scale=None, nlimbs=None):
        pt = self.pt()
        if slots is None and scale is None and nlimbs is None:
            self.ecd(pt, z)
        else:
            self.ecd_ex(pt, z, slots or self.slots, scale or self.info.delta, nlimbs or self.L)
        ct = self.ct()
        self.enc_pk(ct, pt, pk)
        self.free(pt)
        return ct

    def decrypt(self, ct, sk, slots=None):
        pt = self.pt()
        self.dec(pt, ct, sk)
        z = self.dcd(pt, slots)
        self.free(pt)
        return z
