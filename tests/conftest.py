import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "tests")):
    if p not in sys.path:
        sys.path.insert(0, p)

REFERENCE = "/root/reference"


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) and runs the HIP path")


@pytest.fixture(scope="session")
def cuda():
    import torch
    if not torch.cuda.is_available():
        pytest.fail("gpu test run without a visible HIP device")
    import webp_amd
    webp_amd.device_check()
    return torch.device("cuda:0")


_HIP = None


def _hip():
    """The HIP runtime torch already loaded (raw calls for the drain probe)."""
    global _HIP
    if _HIP is None:
        import ctypes
        _HIP = ctypes.CDLL("libamdhip64.so")
        _HIP.hipGetErrorName.restype = ctypes.c_char_p
    return _HIP


@pytest.fixture(autouse=True)
def _gpu_drain(request):
    """After every GPU test, wait for ALL the device's work (every stream)
    and surface any asynchronous device fault there, so that it is reported
    as the teardown error of the test that launched the faulting work, not by
    a later test's first HIP call (an illegal-address error
    first reported in test_gpu_rescale_large, twice, whose kernel was never
    identified).  The probe is hipDeviceSynchronize plus a fresh hipMalloc /
    hipFree -- a new device allocation is the call that reported the sticky
    error both times, where the stream synchronisations of the tests before it
    had returned success.  WG_DRAIN_SLEEP_MS (diagnostic runs) waits that long
    before the probe, for a fault whose notification lags the kernel's end."""
    yield
    if request.node.get_closest_marker("gpu") is None:
        return
    import ctypes
    import os
    import time

    import torch
    if not torch.cuda.is_available():
        return
    torch.cuda.synchronize()
    ms = float(os.environ.get("WG_DRAIN_SLEEP_MS", "0"))
    if ms > 0:
        time.sleep(ms / 1e3)
    hip = _hip()
    rc_sync = hip.hipDeviceSynchronize()
    p = ctypes.c_void_p()
    rc_malloc = hip.hipMalloc(ctypes.byref(p), ctypes.c_size_t(1 << 21))
    if rc_malloc == 0:
        hip.hipFree(p)
    if rc_sync or rc_malloc:
        names = [hip.hipGetErrorName(rc).decode() for rc in (rc_sync, rc_malloc)]
        pytest.fail(f"device error after {request.node.nodeid}: hipDeviceSynchronize -> {names[0]}, "
                    f"hipMalloc -> {names[1]}")
