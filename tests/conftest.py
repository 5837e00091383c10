import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through libtadpole_hip.so)")


@pytest.fixture(scope="session")
def lib():
    from tadpole_amd import _lib
    return _lib.load()


@pytest.fixture(scope="session")
def gpu(lib):
    if lib.tp_device_count() < 1:
        pytest.fail("no HIP device: gpu-marked tests must run on the GPU box")
    return lib
