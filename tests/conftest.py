import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP kernels through the C-ABI)")
    config.addinivalue_line("markers", "slow: larger sizes")


def _gpu_available() -> bool:
    try:
        import ctypes

        hip = ctypes.CDLL("libamdhip64.so")
        n = ctypes.c_int(0)
        return hip.hipGetDeviceCount(ctypes.byref(n)) == 0 and n.value > 0
    except OSError:
        return False


@pytest.fixture(scope="session")
def handle():
    if not _gpu_available():
        pytest.skip("no GPU visible")
    from xerus_amd import capi

    h = capi.Handle(0)
    yield h
    h.close()


@pytest.fixture(scope="session")
def ref():
    from oracle import xerus_ref

    return xerus_ref


@pytest.fixture(scope="session")
def xe():
    """The C++ host API (pybind module over libxerus_amd); GPU only."""
    if not _gpu_available():
        pytest.skip("no GPU visible")
    import xerus_amd.xerus as module

    module.seed(0xBAADF00D)
    return module
