import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if REPO not in sys.path:
    sys.path.insert(0, REPO)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (HIP kernels)")
    config.addinivalue_line("markers", "slow: long-running")


@pytest.fixture(scope="session")
def cme():
    import cme213x

    return cme213x


@pytest.fixture(scope="session")
def gpu():
    import torch

    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import cme213x

    cme213x._ext.hip()  # must load: fail loudly on a GPU box
    return torch.device("cuda:0")


@pytest.fixture(scope="session")
def tune_lib(gpu):
    """The tuning-arm library (libcme213_tune.so: `make TUNE=1` / CME_TUNE=1).
    Not part of the production build, so its arm tests skip without it."""
    import cme213x

    if not (cme213x._ext._LIB_DIR / "libcme213_tune.so").exists():
        pytest.skip("tuning library not built (make TUNE=1)")
    cme213x._ext._load("tune")
    return True
