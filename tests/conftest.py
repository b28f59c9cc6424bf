import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

GOLDEN = os.path.join(ROOT, "tests", "golden")
CONFIGS = os.path.join(GOLDEN, "configs")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (runs the HIP kernels)")
    config.addinivalue_line("markers", "slow: full-size parity case (seconds of oracle time)")


@pytest.fixture(scope="session")
def oracle():
    from oracle import pyoracle
    pyoracle.lib()
    return pyoracle


@pytest.fixture(scope="session")
def mvsv():
    import mvstereovision3_amd
    return mvstereovision3_amd


@pytest.fixture(scope="session")
def gpu():
    """The HIP path must be present on a GPU box: fail loudly, never skip/fallback."""
    import torch
    assert torch.cuda.is_available(), "gpu test selected but no HIP device visible"
    from mvstereovision3_amd import _lib
    _lib.lib()
    return torch
