"""CSTR closed-loop harness: a numpy restatement of HECTR's callers of the
GPQHE API, so the engine can be driven exactly as ``test-hectr cstr-hempc``
drives it, on a GPU box where the reference C sources do not exist.

Restated (behaviour, not code) from /root/reference:
  plant        src/cstr.c:28-132  (cstr_ode, cstr_jacobian, cstr_linearize)
  integrator   src/ode.c:65-95    (ode15s, linearly implicit Euler)
  c2d / expm   src/ctr.c:28-48, src/matrices.c:93-122 (eigen-decomposition expm)
  estimator    src/ctr.c:62-119, src/dlqe.c:39-77, src/dare.c:38-135
  selector     src/ctr.c:121-154, 231-280
  loop         src/ctr.c:363-443 (ctr_simulate, plaintext MPC)
               src/ctr.c:500-618 (hectr_simulate, encrypted MPC)
  MPC          src/mpc.c:113-196, 380-420 (plaintext), src/hempc.c:27-274
  test driver  tests/hectr.c:699-819 (test_cstr_mpc / test_cstr_hempc)

Quirks kept on purpose because the committed fixtures contain them:
  * ctr_measure multiplies C[i][j] by x[i] (not x[j]) (src/ctr.c:156-164);
  * the c2d block matrix has eps(1) in its whole lower half (src/ctr.c:39-42);
  * horizon = N/10 and slots = 2^ceil(log2(nu*horizon + 1)) (src/ctr.c:510-511).

LAPACK calls go through scipy.linalg.lapack with the same routines the
reference uses (zgeev, zgetrf/zgetri, dgetrf/dgetri) so that the eigen-based
expm of the nearly defective c2d matrix is reproduced.
"""
from __future__ import annotations

import math
import time

import numpy as np
from scipy.linalg import lapack

# --- plant parameters (src/cstr.c:26-38) ---------------------------------
RHO, CP, DELTAH, EOVERR, K0, U_HT, C0, T0, RAD = (
    1000.0, 0.239, -5e4, 8750.0, 7.2e10, 54.94, 1.0, 350.0, 0.219)
# steady state (tests/hectr.c: cs, Ts, hs, Tcs, Fs, F0s)
CS, TS, HS, TCS, FS, F0S = 0.878, 324.5, 0.659, 300.0, 0.1, 0.1
HECTR_TOLERANCE, HECTR_SMALL, HECTR_ITER_MAX = 1e-10, 1e-5, 10000

REC = np.dtype([("k", "<u4"), ("x", "<f8", 3), ("u", "<f8", 2)])


def cstr_ode(x, u, p):
    c, T, h = x
    Tc, F = u
    F0 = p[0]
    kT = K0 * math.exp(-EOVERR / T)
    S = math.pi * RAD * RAD
    return np.array([
        F0 * (C0 - c) / (S * h) - kT * c,
        F0 * (T0 - T) / (S * h) + -DELTAH / (RHO * CP) * kT * c + 2 * U_HT / (RAD * RHO * CP) * (Tc - T),
        (F0 - F) / S])


def cstr_jacobian(x, u, p):
    c, T, h = x
    F0 = p[0]
    kT = K0 * math.exp(-EOVERR / T)
    S = math.pi * RAD * RAD
    return np.array([
        [-F0 / (S * h) - kT, -kT * EOVERR / (T * T) * c, -F0 * (C0 - c) / (S * h * h)],
        [(-DELTAH) / (RHO * CP) * kT,
         -F0 / (S * h) + (-DELTAH) / (RHO * CP) * kT * EOVERR / (T * T) * c + -2 * U_HT / (RAD * RHO * CP),
         -F0 * (T0 - T) / (S * h * h)],
        [0.0, 0.0, 0.0]])


def _dinv(a):
    lu, piv, info = lapack.dgetrf(np.asarray(a, dtype=np.float64))
    assert info == 0
    inv, info = lapack.dgetri(lu, piv)
    assert info == 0
    return inv


def _zinv(a):
    lu, piv, info = lapack.zgetrf(np.asarray(a, dtype=np.complex128))
    assert info == 0
    inv, info = lapack.zgetri(lu, piv)
    assert info == 0
    return inv


def dexpm(a):
    """expm by eigen-decomposition, as src/matrices.c:93-122."""
    w, _vl, v, info = lapack.zgeev(np.asarray(a, dtype=np.complex128), compute_vl=0, compute_vr=1)
    assert info == 0
    vd = v * np.exp(w)[None, :]
    return np.real(vd @ _zinv(v))


def eps(a):
    a = abs(a)
    return float(np.nextafter(a, np.inf) - a)


def ctr_c2d(jacA, dt):
    n = jacA.shape[0]
    Cm = np.zeros((2 * n, 2 * n))
    Cm[:n, :n] = jacA * dt
    for i in range(n):
        Cm[i, n + i] = dt
    Cm[n:, :] = eps(1.0)
    e = dexpm(Cm)
    return e[:n, :n].copy(), e[:n, n:].copy()


def cstr_linearize(xs, us, ps, dt):
    c, T, h = xs
    S = math.pi * RAD * RAD
    jacA = cstr_jacobian(xs, us, ps)
    jacB = np.array([[0.0, 0.0], [2 * U_HT / (RAD * RHO * CP), 0.0], [0.0, -1 / S]])
    jacBp = np.array([[(C0 - c) / (S * h)], [(T0 - T) / (S * h)], [1 / S]])
    A, eB = ctr_c2d(jacA, dt)
    return A, eB @ jacB, eB @ jacBp


def ode15s(x, u, p, dt):
    J = cstr_jacobian(x, u, p)
    Cm = np.eye(3) - J * dt
    return x + dt * (_dinv(Cm) @ cstr_ode(x, u, p))


def dare(A, B, Q, R):
    X = Q.copy()
    for _ in range(HECTR_ITER_MAX):
        ATX = A.T @ X
        ATXA = ATX @ A
        ATXB = ATX @ B
        BTX = B.T @ X
        BTXA = BTX @ A
        BTXB = BTX @ B
        inv = _dinv(R + BTXB)
        Xn = ATXA - (ATXB @ inv) @ BTXA + Q
        diff = np.abs(Xn - X).max()
        X = Xn
        if diff < HECTR_TOLERANCE:
            break
    return X


def dlqe(A, Cm, Q, R):
    X = dare(A.T, Cm.T, Q, R)
    XCT = X @ Cm.T
    return XCT @ _dinv(Cm @ XCT + R)


def ctr_estimator(A, B, Cm, Bd, Cd, xs):
    nx, nd, ny = A.shape[0], Bd.shape[1], Cm.shape[0]
    na = nx + nd
    Aaug = np.zeros((na, na))
    Aaug[:nx, :nx] = A
    Aaug[:nx, nx:] = Bd
    Aaug[nx:, nx:] = np.eye(nd)
    Caug = np.zeros((ny, na))
    Caug[:, :nx] = Cm
    Caug[:, ny:ny + nd] = Cd  # src/ctr.c:96-98 indexes Cd at column ny + j
    Qw = np.eye(na) * HECTR_SMALL
    Qw[-1, -1] = 1.0
    Rv = np.diag([HECTR_SMALL * v * v for v in xs])
    L = dlqe(Aaug, Caug, Qw, Rv)
    return L[:nx].copy(), L[nx:].copy()


def ctr_selector(A, B, Cm, H):
    nx, nu = B.shape
    G = np.zeros((nx + nu, nx + nu))
    G[:nx, :nx] = np.eye(nx) - A
    G[:nx, nx:] = -B
    G[nx:, :nx] = H @ Cm
    return _dinv(G)


def calc_horizon_matrices(A, B, Cm, Q, R, N):
    """src/hempc.c:27-95 (same algebra in src/mpc.c)."""
    n, m = B.shape
    l = Cm.shape[0]
    AA = np.zeros((n * (N + 1), n))
    BB = np.zeros((n * (N + 1), m))
    Theta = np.zeros((n * (N + 1), m * N))
    CC = np.zeros((l * (N + 1), n * (N + 1)))
    QQ = np.zeros((l * (N + 1), l * (N + 1)))
    RR = np.zeros((m * N, m * N))
    An = np.eye(n)
    AA[:n] = An
    QQ[:l, :l] = Q
    RR[:m, :m] = R
    CC[:l, :n] = Cm
    for k in range(1, N + 1):
        AnB = An @ B
        BB[k * n:(k + 1) * n] = BB[(k - 1) * n:k * n] + AnB
        An = An @ A
        AA[k * n:(k + 1) * n] = An
        for i in range(k, N + 1):
            Theta[i * n:(i + 1) * n, (i - k) * m:(i - k + 1) * m] = BB[k * n:(k + 1) * n]
        QQ[k * l:(k + 1) * l, k * l:(k + 1) * l] = Q
        if k < N:
            RR[k * m:(k + 1) * m, k * m:(k + 1) * m] = R
        CC[k * l:(k + 1) * l, k * n:(k + 1) * n] = Cm
    return AA, BB, Theta, CC, QQ, RR


def mpc_gains(A, B, Cm, Q, R, N):
    """M_A = H^-1 Theta^T CC^T QQ CC AA, M_B likewise (src/hempc.c:117-196)."""
    AA, BB, Theta, CC, QQ, RR = calc_horizon_matrices(A, B, Cm, Q, R, N)
    CCTheta = CC @ Theta
    TQ = CCTheta.T @ QQ
    H = TQ @ CCTheta + RR
    Hinv = _dinv(H)
    MA = Hinv @ (TQ @ (CC @ AA))
    MB = Hinv @ (TQ @ (CC @ BB))
    return MA, MB, dict(AA=AA, BB=BB, CC=CC, TQ=TQ, Hinv=Hinv)


def d2z_matrix(M, slots):
    """src/matrices.c:133-141: row-major into a slots x slots complex matrix."""
    Z = np.zeros((slots, slots), dtype=np.complex128)
    Z[:M.shape[0], :M.shape[1]] = M
    return Z


def d2z_vector(v, slots):
    z = np.zeros(slots, dtype=np.complex128)
    z[:len(v)] = v
    return z


class CstrProblem:
    """Fixed setup of test_cstr_mpc / test_cstr_hempc (tests/hectr.c:699-805)."""

    def __init__(self, N=40):
        self.nx, self.nu, self.np_, self.ny, self.nd = 3, 2, 1, 3, 2
        self.xs = np.array([CS, TS, HS])
        self.us = np.array([TCS, FS])
        self.ps = np.array([F0S])
        self.dt = 1.0
        self.A, self.B, self.Bp = cstr_linearize(self.xs, self.us, self.ps, self.dt)
        self.C = np.eye(3)
        self.Bd = np.zeros((3, 2))
        self.Cd = np.array([[1.0, 0.0], [0.0, 0.0], [0.0, 1.0]])
        self.Hr = np.array([[1.0, 0.0, 0.0], [0.0, 0.0, 1.0]])
        self.N = N
        self.p = np.zeros(N)
        self.p[9:] = 0.1 * F0S
        self.horizon = N // 10
        self.slots = 1 << (32 - _clz32(self.nu * self.horizon))
        self.Q = np.diag(1.0 / self.xs ** 2)
        self.R = np.diag(1.0 / self.us ** 2)
        self.Lx, self.Ld = ctr_estimator(self.A, self.B, self.C, self.Bd, self.Cd, self.xs)
        self.Ginv = ctr_selector(self.A, self.B, self.C, self.Hr)
        self.MA, self.MB, self._mpc = mpc_gains(self.A, self.B, self.C, self.Q, self.R, self.horizon)

    def regulator_plain(self, xhat, uhat, xr, ur):
        """ctr_mpc without constraints (src/mpc.c:380-420): e, c, du = -H^-1 c,
        u = uhat + du[:m] (calc_u's cumulative sum is du for the first m)."""
        g = self._mpc
        e = g["CC"] @ (g["AA"] @ (xhat - xr) + g["BB"] @ (uhat - ur))
        c = g["TQ"] @ e
        du = g["Hinv"] @ (-c)
        return uhat + du[:self.nu]

    def simulate(self, regulator, on_step=None):
        """Closed loop of src/ctr.c:571-595 (both ctr_simulate and
        hectr_simulate share it; only the control law differs)."""
        nx, nu, nd, N = self.nx, self.nu, self.nd, self.N
        x = np.zeros((N + 1, nx))
        u = np.zeros((N, nu))
        xhatm = np.zeros(nx)
        dhatm = np.zeros(nd)
        rsp = np.zeros(nu)
        Csum = self.C.sum(axis=1)
        for k in range(N + 1):
            y = Csum * x[k]                                  # ctr_measure quirk
            e = y - self.C @ xhatm - self.Cd @ dhatm        # ctr_measure_forward
            xhat = xhatm + self.Lx @ e
            dhat = dhatm + self.Ld @ e
            if k == N:
                break
            pack = np.concatenate([self.Bd @ dhat, rsp - self.Hr @ (self.Cd @ dhat)])
            r = self.Ginv @ pack                             # ctr_select
            xr, ur = r[:nx], r[nx:]
            if k == 0:
                u[0] = ur
            uhat = (u[0] if k == 0 else u[k - 1]).copy()
            u[k] = regulator(xhat, uhat, xr, ur)
            if on_step:
                on_step(k, xhat, uhat, xr, ur, u[k])
            xx = x[k] + self.xs                              # ctr_actuate
            uu = u[k] + self.us
            pp = np.array([self.p[k]]) + self.ps
            for _ in range(2):
                xx = ode15s(xx, uu, pp, self.dt / 2)
            x[k + 1] = xx - self.xs
            xhatm = self.A @ xhat + self.B @ u[k] + self.Bd @ dhat   # ctr_estimate
            dhatm = dhat
        return x + self.xs, u + self.us

    @staticmethod
    def records(x, u):
        """The 41 x 44-byte records of tests/hectr.c:751-756 / 812-817."""
        N = u.shape[0]
        rec = np.zeros(N + 1, dtype=REC)
        rec["k"] = np.arange(N + 1)
        rec["x"] = x
        rec["u"][:N] = u
        rec["u"][N] = u[N - 1]
        return rec


def _clz32(v):
    return 32 - int(v).bit_length()


class EncryptedRegulator:
    """hectr_enc_states -> ctr_hempc -> hectr_dec_state (src/ctr.c:445-498,
    src/hempc.c:216-274), issuing the same he_* calls in the same order."""

    def __init__(self, engine, problem: CstrProblem, logn=12, logq=109, log_delta=50, seed=None,
                 init=True):
        self.e = engine
        self.pb = problem
        if init:
            engine.init(logn, logq, problem.slots, log_delta)
        if seed is not None:
            engine.set_seed(seed)
        s = problem.slots
        self.pk, self.sk = engine.pk(), engine.sk()
        self.rk = engine.evks(s)
        t0 = time.perf_counter()
        engine.keypair(self.pk, self.sk)
        engine.genrk(self.rk, self.sk)
        engine.sync()
        self.keygen_s = time.perf_counter() - t0
        self.ct = {k: engine.ct() for k in ("xhat", "uhat", "xr", "ur", "up")}
        self.MAz = d2z_matrix(problem.MA, s).ravel()
        self.MBz = d2z_matrix(problem.MB, s).ravel()
        self.timings = []

    def __call__(self, xhat, uhat, xr, ur):
        e, s, c = self.e, self.pb.slots, self.ct
        t0 = time.perf_counter()
        # hectr_enc_states (src/ctr.c:445-481): encode + encrypt 5 vectors
        vals = {"up": np.zeros(s), "xhat": xhat, "uhat": uhat, "xr": xr, "ur": ur}
        pts = {k: e.pt() for k in ("up", "xhat", "uhat", "xr", "ur")}  # src/ctr.c:461-465
        for k in ("up", "xhat", "uhat", "xr", "ur"):
            e.ecd(pts[k], d2z_vector(vals[k], s))
        for k in ("up", "xhat", "uhat", "xr", "ur"):
            e.enc_pk(c[k], pts[k], self.pk)
        for k in pts:
            e.free(pts[k])
        # ctr_hempc (src/hempc.c:240-273)
        xdiff, udiff, du, uhat_copy, MAx, MBu = (e.ct() for _ in range(6))
        e.sub(xdiff, c["xhat"], c["xr"])
        e.sub(udiff, c["uhat"], c["ur"])
        e.gemv(MAx, self.MAz, xdiff, self.rk)
        e.gemv(MBu, self.MBz, udiff, self.rk)
        e.add(du, MAx, MBu)
        e.neg(du)
        e.copy_ct(uhat_copy, c["uhat"])
        e.moddown(uhat_copy)
        e.add(c["up"], uhat_copy, du)
        for o in (xdiff, udiff, du, uhat_copy, MAx, MBu):
            e.free(o)
        # hectr_dec_state (src/ctr.c:483-498)
        pt = e.pt()
        e.dec(pt, c["up"], self.sk)
        uz = e.dcd(pt)
        e.free(pt)
        assert np.all(uz.imag < HECTR_SMALL), "imaginary part too large (src/ctr.c:493-494)"
        self.timings.append(time.perf_counter() - t0)
        return uz.real[:self.pb.nu].copy()

    def close(self):
        e = self.e
        for o in self.ct.values():
            e.free(o)
        e.free(self.pk)
        e.free(self.sk)
        e.free_evks(self.rk)
