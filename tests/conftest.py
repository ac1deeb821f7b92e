"""pytest configuration: the `gpu` marker and shared engine fixtures.

`-m "not gpu"` runs on the CPU container (oracle vs model / fixtures, ABI
loading, host logic); `-m gpu` runs on an MI355X and compares the product
library against the oracle bit for bit.
"""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device) and the product library")


@pytest.fixture(scope="session")
def oracle():
    from hectr_amd.gpqhe import Engine
    return Engine.oracle()


@pytest.fixture(scope="session")
def product():
    import torch
    if not torch.cuda.is_available():
        pytest.fail("gpu test without a visible HIP device")
    from hectr_amd.gpqhe import Engine
    return Engine.product()
