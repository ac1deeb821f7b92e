"""harness/lapacke_subset.c (liblapacke.so: the six LAPACKE routines HECTR's
controller code calls, reference src/matrices.c:43-99) checked directly, by
residuals, on random, structured, wide/tall, singular and defective inputs --
not only through the CSTR trajectory.  Where SciPy is importable its bundled
OpenBLAS LAPACKE (scipy_LAPACKE_*) is called on the same inputs as a second
opinion on the return codes."""
import ctypes
import glob
import os

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "harness", "lib", "liblapacke.so")
ROW, COL = 101, 102
dp = np.ctypeslib.ndpointer(dtype=np.float64, flags="C_CONTIGUOUS")
zp = np.ctypeslib.ndpointer(dtype=np.complex128, flags="C_CONTIGUOUS")
ip = np.ctypeslib.ndpointer(dtype=np.int32, flags="C_CONTIGUOUS")


def _bind(lib, prefix=""):
    f = {}
    c_int, c_char = ctypes.c_int, ctypes.c_char
    f["dgetrf"] = getattr(lib, prefix + "LAPACKE_dgetrf")
    f["dgetrf"].argtypes = [c_int, c_int, c_int, dp, c_int, ip]
    f["dgetri"] = getattr(lib, prefix + "LAPACKE_dgetri")
    f["dgetri"].argtypes = [c_int, c_int, dp, c_int, ip]
    f["zgetrf"] = getattr(lib, prefix + "LAPACKE_zgetrf")
    f["zgetrf"].argtypes = [c_int, c_int, c_int, zp, c_int, ip]
    f["zgetri"] = getattr(lib, prefix + "LAPACKE_zgetri")
    f["zgetri"].argtypes = [c_int, c_int, zp, c_int, ip]
    f["dgesvd"] = getattr(lib, prefix + "LAPACKE_dgesvd")
    f["dgesvd"].argtypes = [c_int, c_char, c_char, c_int, c_int, dp, c_int, dp, dp, c_int, dp, c_int, dp]
    f["zgeev"] = getattr(lib, prefix + "LAPACKE_zgeev")
    f["zgeev"].argtypes = [c_int, c_char, c_char, c_int, zp, c_int, zp, ctypes.c_void_p, c_int, zp, c_int]
    for fn in f.values():
        fn.restype = c_int
    return f


@pytest.fixture(scope="module")
def lap():
    if not os.path.exists(LIB):
        import subprocess
        subprocess.run(["make", "-C", os.path.join(ROOT, "harness")], check=True, capture_output=True)
    return _bind(ctypes.CDLL(LIB))


@pytest.fixture(scope="module")
def openblas():
    try:
        import scipy
    except ImportError:
        pytest.skip("SciPy absent")
    libs = glob.glob(os.path.join(os.path.dirname(scipy.__file__), "..", "scipy.libs", "libscipy_openblas*.so"))
    if not libs:
        pytest.skip("SciPy's OpenBLAS not found")
    return _bind(ctypes.CDLL(libs[0]), "scipy_")


def inverse(f, A, cplx=False):
    n = A.shape[0]
    a = np.ascontiguousarray(A.astype(np.complex128 if cplx else np.float64))
    piv = np.zeros(n, dtype=np.int32)
    e1 = f["zgetrf" if cplx else "dgetrf"](ROW, n, n, a, n, piv)
    if e1:
        return e1, None
    e2 = f["zgetri" if cplx else "dgetri"](ROW, n, a, n, piv)
    return e2, a


def matrices(rng):
    yield "random", rng.standard_normal((6, 6))
    yield "ill", np.vander(np.linspace(1, 2, 5), increasing=True)  # cond ~ 1e6
    yield "permuted", np.eye(7)[rng.permutation(7)] * 3 + 0.01 * rng.standard_normal((7, 7))
    yield "one", np.array([[4.0]])


@pytest.mark.parametrize("cplx", [False, True])
def test_getrf_getri_inverse(lap, cplx):
    rng = np.random.default_rng(1)
    for name, A in matrices(rng):
        if cplx:
            A = A + 1j * rng.standard_normal(A.shape)
        err, Ai = inverse(lap, A, cplx)
        assert err == 0, name
        r = np.abs(A @ Ai - np.eye(len(A))).max()
        assert r < 1e-9 * np.linalg.cond(A), (name, r)


def test_getrf_singular(lap, openblas):
    """A zero pivot: info = its 1-based index, as LAPACK reports it."""
    A = np.array([[1.0, 2, 3], [2, 4, 6], [1, 0, 1]])
    for f in (lap, openblas):
        a = A.copy()
        piv = np.zeros(3, dtype=np.int32)
        info = f["dgetrf"](ROW, 3, 3, a, 3, piv)
        assert info > 0
    a = np.zeros((2, 2))
    assert lap["dgetrf"](ROW, 2, 2, a, 2, np.zeros(2, dtype=np.int32)) == 1


@pytest.mark.parametrize("m,n", [(4, 4), (3, 6), (6, 3), (5, 1), (1, 4)])
@pytest.mark.parametrize("layout", [ROW, COL])
def test_dgesvd_full(lap, m, n, layout):
    rng = np.random.default_rng(m * 10 + n)
    for A in (rng.standard_normal((m, n)), np.outer(rng.standard_normal(m), rng.standard_normal(n))):  # rank 1 too
        order = "C" if layout == ROW else "F"
        a = np.ascontiguousarray(A) if layout == ROW else np.asfortranarray(A)
        buf = np.ascontiguousarray(a.ravel(order="K"))
        s = np.zeros(min(m, n))
        u = np.zeros(m * m)
        vt = np.zeros(n * n)
        sup = np.zeros(max(1, min(m, n) - 1))
        lda = n if layout == ROW else m
        info = lap["dgesvd"](layout, b"A", b"A", m, n, buf, lda, s, u, m, vt, n, sup)
        assert info == 0
        U = u.reshape((m, m), order=order)
        VT = vt.reshape((n, n), order=order)
        S = np.zeros((m, n))
        S[:len(s), :len(s)] = np.diag(s)
        assert np.abs(U @ S @ VT - A).max() < 1e-12 * max(1, np.abs(A).max())
        assert np.abs(U.T @ U - np.eye(m)).max() < 1e-12
        assert np.abs(VT @ VT.T - np.eye(n)).max() < 1e-12
        assert np.all(np.diff(s) <= 1e-15) and np.all(s >= 0)
        assert np.allclose(s, np.linalg.svd(A, compute_uv=False), rtol=1e-12, atol=1e-13)


def eig(f, A):
    n = len(A)
    a = np.ascontiguousarray(A.astype(np.complex128))
    w = np.zeros(n, dtype=np.complex128)
    vr = np.zeros(n * n, dtype=np.complex128)
    info = f["zgeev"](ROW, b"N", b"V", n, a, n, w, None, n, vr, n)
    return info, w, vr.reshape(n, n)


def test_zgeev_eigenpairs(lap, openblas):
    rng = np.random.default_rng(3)
    cases = {
        "random": rng.standard_normal((6, 6)) + 1j * rng.standard_normal((6, 6)),
        "real_nonsym": rng.standard_normal((5, 5)),  # complex-conjugate pairs
        "repeated": np.diag([2.0, 2.0, 2.0, -1.0]) + 0j,
        "defective": np.array([[3.0, 1, 0], [0, 3, 1], [0, 0, 3]]) + 0j,  # one Jordan block
        "cstr_like": np.array([[0.9, 0.1, 0], [-0.05, 0.95, 0.02], [0, 0, 1.0]]) + 0j,
        "zero": np.zeros((3, 3), dtype=np.complex128),
    }
    for name, A in cases.items():
        info, w, V = eig(lap, A)
        assert info == 0, name
        # residual per eigenpair, unit-norm columns
        for k in range(len(A)):
            v = V[:, k]
            assert abs(np.linalg.norm(v) - 1) < 1e-12, name
            assert np.abs(A @ v - w[k] * v).max() < 1e-9 * max(1, np.abs(A).max()), name
        # eigenvalues agree with OpenBLAS's as multisets (defective: to the
        # accuracy a Jordan block allows, ~eps^(1/3))
        _, wo, _ = eig(openblas, A)
        tol = 1e-4 if name == "defective" else 1e-10
        got, want = np.sort_complex(w), np.sort_complex(wo)
        assert np.abs(got - want).max() < tol * max(1, np.abs(want).max()), name
