import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)
TESTS = os.path.dirname(os.path.abspath(__file__))
if TESTS not in sys.path:
    sys.path.insert(0, TESTS)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device); run with -m gpu")
    config.addinivalue_line("markers", "slow: long-running")


def gpu_available() -> bool:
    try:
        import torch

        return torch.cuda.is_available()
    except Exception:
        return False


@pytest.fixture(scope="session")
def oracle():
    import oracle_lib

    oracle_lib.build()
    return oracle_lib


@pytest.fixture(autouse=True)
def _no_ring_faults(request):
    """After every GPU test that used the codec in this process: no kernel's
    loader-ring handshake hit its spin cap (codec_device.h ring_sweep; a
    capped spin means wrong outputs, so it fails the test loudly)."""
    yield
    if request.node.get_closest_marker("gpu") is None:
        return
    import redset_amd._lib as L

    if L._lib is None or not gpu_available():
        return
    import redset_amd

    assert redset_amd.ring_faults() == 0, "a loader-ring handshake hit its spin cap"
