"""End-to-end parity against the reference's own committed closed-loop runs
(tests/golden/cstr-*.bin, written by reference tests/hectr.c:751-756,
812-817, 821-847).  CPU: the numpy restatement of HECTR's plaintext loop and
the oracle engine behind the encrypted regulator.  The GPU version of the
encrypted loop lives in tests/test_gpu_cstr.py."""
import os

import numpy as np
import pytest

from hectr_amd.cstr import REC, CstrProblem, EncryptedRegulator

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def load(name):
    with open(os.path.join(GOLD, name + ".bin"), "rb") as f:
        return np.frombuffer(f.read(), dtype=REC)


def rel(a, b):
    return float(np.max(np.abs(a - b) / np.abs(b).clip(1e-300)))


def test_fixture_self_consistency():
    """cstr-cmp.bin is exactly |cstr-mpc - cstr-hempc| (tests/hectr.c:835-843)."""
    mpc, hempc, cmp_ = load("cstr-mpc"), load("cstr-hempc"), load("cstr-cmp")
    assert np.array_equal(cmp_["x"], np.abs(mpc["x"] - hempc["x"]))
    assert np.array_equal(cmp_["u"], np.abs(mpc["u"] - hempc["u"]))
    assert rel(hempc["x"], mpc["x"]) < 2e-11 and rel(hempc["u"], mpc["u"]) < 2e-11


def test_plaintext_loop_matches_cstr_mpc():
    pb = CstrProblem(40)
    x, u = pb.simulate(pb.regulator_plain)
    rec = pb.records(x, u)
    ref = load("cstr-mpc")
    assert rel(rec["x"], ref["x"]) < 1e-10
    assert rel(rec["u"], ref["u"]) < 1e-10
    # the 6-significant-digit text fixture as well
    txt = np.loadtxt(os.path.join(GOLD, "cstr-mpc.txt"))
    assert np.allclose(txt[:, 1:4], rec["x"], rtol=1e-5, atol=0)
    assert np.allclose(txt[:, 4:6], rec["u"], rtol=1e-5, atol=0)


def test_gain_structure():
    """slots = 16 for nu=2, horizon=4 (src/ctr.c:510-511); M_A has 10 and M_B
    9 non-zero generalized diagonals."""
    pb = CstrProblem(40)
    assert pb.horizon == 4 and pb.slots == 16
    from hectr_amd.cstr import d2z_matrix
    for M, nz in ((pb.MA, 10), (pb.MB, 9)):
        Z = d2z_matrix(M, 16)
        diags = [d for d in range(16) if any(Z[i, (i + d) % 16] != 0 for i in range(16))]
        assert len(diags) == nz


def test_oracle_encrypted_loop_matches_cstr_hempc(oracle):
    """HECTR's own parameters: hectx_init(12, 2^109, 16, 2^50)."""
    pb = CstrProblem(40)
    reg = EncryptedRegulator(oracle, pb, seed=7)
    x, u = pb.simulate(reg)
    reg.close()
    rec = pb.records(x, u)
    for name in ("cstr-hempc", "cstr-mpc"):
        ref = load(name)
        assert rel(rec["x"], ref["x"]) < 1e-9, name
        assert rel(rec["u"], ref["u"]) < 1e-9, name


@pytest.mark.parametrize("seed", [1, 99])
def test_oracle_config1_n8192_l4(oracle, seed, monkeypatch):
    """BASELINE config 1: the unchanged caller with N=2^13, L=4 through the
    environment override of hectx_init (GPQHE_LOGN / GPQHE_NLIMBS)."""
    monkeypatch.setenv("GPQHE_LOGN", "13")
    monkeypatch.setenv("GPQHE_NLIMBS", "4")
    pb = CstrProblem(40)
    pb.N = 12  # bounded sample of the 40-step loop keeps the CPU suite fast
    reg = EncryptedRegulator(oracle, pb, seed=seed)
    assert oracle.n == 8192 and oracle.L == 4
    x, u = pb.simulate(reg)
    reg.close()
    ref = load("cstr-mpc")[:pb.N + 1]
    rec = pb.records(x, u)
    assert rel(rec["x"][:pb.N], ref["x"][:pb.N]) < 1e-6
    assert rel(rec["u"][:pb.N], ref["u"][:pb.N]) < 1e-6
