import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(ROOT, "oxidized-mtbl_amd"), os.path.join(ROOT, "oracle"), ROOT):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a gfx950 GPU (runs on the MI355X box)")


@pytest.fixture(scope="session")
def oracle():
    import pyoracle
    pyoracle.build()
    return pyoracle


@pytest.fixture(scope="session")
def mtblx_lib():
    import mtblx
    return mtblx.lib()


@pytest.fixture(autouse=True)
def _sync_after_gpu_test(request):
    """GPU tests end with a device synchronize, so an asynchronous fault is reported by the test
    whose launches caused it, not by the next test's first copy"""
    yield
    if request.node.get_closest_marker("gpu") is None or "torch" not in sys.modules:
        return
    import torch
    if torch.cuda.is_available() and torch.cuda.is_initialized():
        torch.cuda.synchronize()
