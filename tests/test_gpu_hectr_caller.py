"""N1 on the MI355X: the unchanged HECTR harness binary (built in the CPU
container from /root/reference by `make -C harness hectr`, see
tests/test_hectr_caller.py) runs `test-hectr cstr-hempc` against the product
libgpqhe.so (hectr_amd/lib).  Its decoded trajectory must match the
reference's plaintext run within 1e-6 relative and equal the same binary's
run on the CPU oracle bit for bit (same seed, bit-exact engine)."""
import os

import numpy as np
import pytest

from tests.test_hectr_caller import OUT, ROOT, compare_to_mpc, run_cstr_hempc

pytestmark = pytest.mark.gpu

BIN = os.path.join(OUT, "test-hectr")


@pytest.mark.skipif(not os.path.exists(BIN), reason="harness binary not built (make -C harness hectr needs the "
                                                      "reference sources, present only in the build container)")
def test_cstr_hempc_unchanged_on_mi355x(tmp_path, product):
    rec, ms = run_cstr_hempc(os.path.join(ROOT, "hectr_amd", "lib"), tmp_path / "gpu")
    dev = compare_to_mpc(rec)
    assert dev < 1e-6, dev
    ora, _ = run_cstr_hempc(os.path.join(OUT, "cpu"), tmp_path / "cpu")
    assert np.array_equal(rec, ora), "GPU and oracle trajectories differ"
    print(f"unchanged test-hectr cstr-hempc on MI355X: 40 steps in {ms} ms (harness pmu timer), "
          f"max rel dev vs cstr-mpc.bin {dev:.2e}")


DRIVER = os.path.join(OUT, "cstr-run")


@pytest.mark.skipif(not os.path.exists(DRIVER), reason="config 4 driver not built (make -C harness hectr, build "
                                                         "container only)")
def test_config4_100_steps_c_caller_on_mi355x(tmp_path, product):
    """Config 4 at its own shape (100 steps, horizon 10, 32 slots) through the
    reference's unchanged hectr_simulate (harness/cstr_run.c) on the MI355X
    library: the trajectory equals the same binary's run on the CPU oracle
    bit for bit.  Against the plaintext fixture both deviate alike: the
    reference's ctr_hempc overflows a 32 x 32 stack matrix at this horizon
    (src/hempc.c:233-234; tests/test_cstr_driver.py pins the overflow-free
    run to 3e-11)."""
    from tests.test_cstr_driver import fixture, rel_dev, run_driver
    (tmp_path / "gpu").mkdir()
    (tmp_path / "cpu").mkdir()
    gpu, ms, _ = run_driver(DRIVER, "hempc", 100, tmp_path / "gpu", os.path.join(ROOT, "hectr_amd", "lib"))
    ora, _, _ = run_driver(DRIVER, "hempc", 100, tmp_path / "cpu", os.path.join(OUT, "cpu"))
    assert np.array_equal(gpu, ora), "GPU and oracle trajectories differ"
    print(f"config 4 C caller on MI355X: 100 steps in {ms} ms (reference pmu timer), "
          f"dev vs cstr-mpc-100.bin {rel_dev(gpu, fixture(100)):.2e} (reference overflow, same on the oracle)")
