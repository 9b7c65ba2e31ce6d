import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through the HIP C-ABI library)")
    config.addinivalue_line("markers", "slow: long-running")


@pytest.fixture(scope="session")
def gpu():
    """Skip-free on the GPU box: a missing device or library is a hard failure there."""
    import torch
    if not torch.cuda.is_available():
        pytest.fail("gpu tests need a visible GPU (they are selected with -m gpu)")
    from recoup_amd import _lib
    _lib.lib()
    return 0
