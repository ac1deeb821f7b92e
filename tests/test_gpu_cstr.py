"""The encrypted CSTR-MPC closed loop (reference test-hectr cstr-hempc,
tests/hectr.c:760-819) driven through the MI355X product library.

* HECTR's own parameters (hectx_init(12, 2^109, 16, 2^50), src/ctr.c:514-518):
  decoded trajectory within 1e-9 relative of the reference's committed
  encrypted run cstr-hempc.bin and of cstr-mpc.bin, and -- same seed --
  bit-identical to the oracle-driven loop (the u values are equal doubles).
* config 4 shape: 100 steps (horizon 10, 32 slots) against the reference's
  own plaintext ctr_simulate at N = 100 (tests/golden/cstr-mpc-100.bin,
  tests/make_cstr_fixture.sh) and the restatement's plaintext loop.
"""
import os

import numpy as np
import pytest

from hectr_amd.cstr import REC, CstrProblem, EncryptedRegulator

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def load(name):
    with open(os.path.join(GOLD, name + ".bin"), "rb") as f:
        return np.frombuffer(f.read(), dtype=REC)


def rel(a, b):
    return float(np.max(np.abs(a - b) / np.abs(b).clip(1e-300)))


def run_loop(engine, N=40, seed=7):
    pb = CstrProblem(N)
    reg = EncryptedRegulator(engine, pb, seed=seed)
    x, u = pb.simulate(reg)
    reg.close()
    return pb, pb.records(x, u), reg


def test_cstr_hempc_on_gpu_matches_fixtures_and_oracle(product, oracle):
    _, rec_p, reg = run_loop(product)
    for name in ("cstr-hempc", "cstr-mpc"):
        ref = load(name)
        assert rel(rec_p["x"], ref["x"]) < 1e-9, name
        assert rel(rec_p["u"], ref["u"]) < 1e-9, name
    _, rec_o, _ = run_loop(oracle)
    assert np.array_equal(rec_p["u"], rec_o["u"]) and np.array_equal(rec_p["x"], rec_o["x"])
    assert np.median(reg.timings) < 0.05  # encrypted regulator step well under 50 ms


def test_cstr_100_steps_on_gpu(product):
    pb = CstrProblem(100)
    assert pb.horizon == 10 and pb.slots == 32
    xp, up = pb.simulate(pb.regulator_plain)
    reg = EncryptedRegulator(product, pb, seed=3)
    x, u = pb.simulate(reg)
    reg.close()
    assert rel(x, xp) < 1e-8 and rel(u, up) < 1e-8
    rec, ref = pb.records(x, u), load("cstr-mpc-100")
    assert rel(rec["x"], ref["x"]) < 1e-6 and rel(rec["u"], ref["u"]) < 1e-6
