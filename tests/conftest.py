import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through the HIP C-ABI)")


@pytest.fixture(scope="session")
def oracle():
    import oracle as orc
    orc.load()
    return orc


@pytest.fixture(scope="session")
def gpu():
    """Fails loudly (never skips) when a gpu-marked test runs without a usable GPU."""
    from raytracingstudy_amd import device_count
    n = device_count()
    assert n > 0, "gpu test but no HIP device visible"
    return n
