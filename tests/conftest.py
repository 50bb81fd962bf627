import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(ROOT, "cpu-renderer_amd"), os.path.join(ROOT, "oracle"), ROOT):
    if p not in sys.path:
        sys.path.insert(0, p)


def _abort_bt_install():
    """Diagnostics (PRK_ABORT_BT=1): a native backtrace on SIGABRT
    (tools/abort_bt.c), installed again at interpreter exit because pytest's
    faulthandler restores the handlers it replaced when the session ends."""
    import ctypes
    lib = os.path.join(ROOT, "tools", "libabort_bt.so")
    if os.path.exists(lib):
        ctypes.CDLL(lib).abort_bt_install()


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through libprk_hip.so on the device)")
    if os.environ.get("PRK_ABORT_BT"):
        import atexit
        import prk  # noqa: F401  (its own exit hook registers first, runs after ours)
        _abort_bt_install()
        atexit.register(_abort_bt_install)


def gpu_available():
    try:
        import prk
        return prk.device_count() > 0
    except Exception:
        return False


@pytest.fixture(scope="session")
def gpu():
    import prk
    n = prk.device_count()  # raises if libprk_hip.so is missing: the HIP path must load
    if n <= 0:
        pytest.fail("gpu-marked test but no HIP device visible")
    return n


@pytest.fixture(autouse=True)
def _hip_last_error_trace(request):
    """Diagnostics (PRK_TRACE_HIP=1): the thread's sticky HIP error after each
    test, so a call that failed silently is pinned to the test that made it."""
    yield
    if not os.environ.get("PRK_TRACE_HIP") or request.node.get_closest_marker("gpu") is None:
        return
    import ctypes
    try:
        hip = ctypes.CDLL("libamdhip64.so")
    except OSError:
        return
    e = hip.hipGetLastError()
    if e:
        hip.hipGetErrorName.restype = ctypes.c_char_p
        sys.stderr.write("PRK_TRACE_HIP: %s left HIP error %d (%s)\n"
                         % (request.node.nodeid, e, hip.hipGetErrorName(e).decode()))
