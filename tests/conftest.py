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
    config.addinivalue_line("markers", "gpu: needs an MI355X (run on the GPU box)")
    config.addinivalue_line("markers", "slow: long-running")


@pytest.fixture(scope="session", autouse=True)
def _built():
    """Build the oracle (and the HIP library when hipcc is present) once per session."""
    from abnn_amd import build

    build.build_oracle()
    if os.path.exists(build.HIPCC):
        build.build_hip()
    yield


@pytest.fixture(scope="session")
def gpu():
    import abnn_amd

    n = abnn_amd.device_count()
    if n == 0:
        pytest.fail("a gpu-marked test ran without a visible HIP device")
    return 0
