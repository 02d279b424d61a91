import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

import __graft_entry__ as ge  # noqa: E402

GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs on the GPU box)")
    config.addinivalue_line("markers", "slow: full-size (10M) parity checks")


@pytest.fixture(scope="session")
def orc():
    """Oracle module (test infrastructure)."""
    return ge.load_oracle()


@pytest.fixture(scope="session")
def oracle(orc):
    return orc.Oracle()


@pytest.fixture(scope="session")
def pkg():
    return ge.load_package()


@pytest.fixture(scope="session")
def dev():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device("cuda:0")


def load_golden(name):
    path = os.path.join(GOLDEN, name)
    if not os.path.exists(path):
        pytest.fail(f"golden fixture {path} missing (run tools/make_golden.py here)")
    with np.load(path, allow_pickle=False) as z:
        return {k: z[k] for k in z.files}


class default_dtype:
    """torch's default dtype set for a block (the reference's statements allocate H with it:
    torch.zeros / torch.ones without a dtype, Modules_Runtime_Test.py:296, :372)."""

    def __init__(self, dt):
        import torch
        self.dt, self.torch = dt, torch

    def __enter__(self):
        self.prev = self.torch.get_default_dtype()
        self.torch.set_default_dtype(self.dt)

    def __exit__(self, *exc):
        self.torch.set_default_dtype(self.prev)

