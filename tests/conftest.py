import os
import sys

import pytest

# torch's own HIP runtime must be loaded before libstorb_rs.so's (see the
# storb_amd/_lib.py docstring); CPU-only test modules may load the library
# first otherwise, and a later torch.cuda call then finds no GPU.
import torch  # noqa: F401  (before any storb_amd import)

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a gfx950 (MI355X) device")
    config.addinivalue_line("markers", "slow: full BASELINE-size cases")


@pytest.fixture(scope="session")
def ctx():
    from storb_amd import _lib
    import torch
    c = _lib.Context(0)
    # Launch on torch's current stream so torch ops in the tests are ordered
    # with the library's kernels.
    c.default_stream = torch.cuda.current_stream(0).cuda_stream
    yield c
    c.close()


@pytest.fixture(autouse=True)
def _device_clean_after_gpu_test(request):
    """After every GPU test, wait for the device: a fault left by that test's
    asynchronous work (queued kernels, async ops, host functions) is then
    reported against it, not against whichever test next touches the GPU."""
    yield
    if request.node.get_closest_marker("gpu") is None:
        return
    import torch
    if torch.cuda.is_available() and torch.cuda.is_initialized():
        torch.cuda.synchronize()
