import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (ROCm GPU); runs the HIP kernels")


@pytest.fixture(scope="session")
def gpu():
    import torch
    if not torch.cuda.is_available():
        pytest.fail("gpu-marked test but no ROCm GPU is visible")
    from omnidirectional_collaborative_filtering_amd import _lib
    _lib.load()
    return torch.device("cuda")


@pytest.fixture
def chunked_encdec(gpu):
    """ocf_gather_encdec in its chunked form for the test (tests comparing launch forms bit for bit against the
    two-launch gathers: the row-resident form sums in another order)"""
    import ctypes
    from omnidirectional_collaborative_filtering_amd import _lib
    prev = ctypes.c_int32()
    _lib.call("ocf_set_tuning", b"encdec_rowres", 0, ctypes.byref(prev))
    yield
    _lib.call("ocf_set_tuning", b"encdec_rowres", prev.value, None)
