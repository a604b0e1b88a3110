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


@pytest.fixture(autouse=True)
def _gpu_drain(request):
    """After every GPU test, wait for ALL the device's work (every stream)
    and surface any asynchronous kernel fault there: a fault is then reported
    as the teardown error of the test that launched the kernel, not by the
    next test's first HIP call (a fault reported in
    test_gpu_rescale_large whose kernel was never identified)."""
    yield
    if request.node.get_closest_marker("gpu") is None:
        return
    import torch
    if torch.cuda.is_available():
        torch.cuda.synchronize()
