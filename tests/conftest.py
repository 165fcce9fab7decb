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


HEARTBEAT_S = 45.0


@pytest.hookimpl(hookwrapper=True)
def pytest_runtest_call(item):
    """A progress line every HEARTBEAT_S seconds while a test runs, written past
    the output capture: the full-size tests (config 4 random mode's eight
    threaded oracle shards, config 5) run minutes without a result line, and
    the GPU box takes a command silent for 3 minutes to be hung."""
    import threading
    import time

    tr = item.config.pluginmanager.get_plugin("terminalreporter")
    capman = item.config.pluginmanager.get_plugin("capturemanager")
    stop = threading.Event()
    t0 = time.monotonic()

    def beat():
        while not stop.wait(HEARTBEAT_S):
            try:  # (the capture is lifted for the one line)
                with capman.global_and_fixture_disabled():
                    tr.write_line(f"  [running {time.monotonic() - t0:.0f} s] {item.nodeid}", flush=True)
            except Exception:
                return

    th = threading.Thread(target=beat, daemon=True) if tr is not None else None
    if th:
        th.start()
    try:
        yield
    finally:
        stop.set()
        if th:
            th.join()


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
