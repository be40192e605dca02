import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(ROOT, "oxidized-mtbl_amd"), os.path.join(ROOT, "oracle"), ROOT):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a gfx950 GPU (runs on the MI355X box)")
    if os.environ.get("MTBLX_POISON"):
        # every uninitialised allocation -- torch.empty here, the library's own
        # scratch through MTBLX_DEBUG_POISON -- is filled with all-ones (0xFF bytes, INT_MAX words)
        # instead of whatever a previous test left, so a kernel whose addressing depends on memory
        # it reads before writing faults or differs deterministically rather than now and then
        os.environ["MTBLX_DEBUG_POISON"] = "1"
        import torch
        import torch.utils.deterministic
        torch.use_deterministic_algorithms(True, warn_only=True)
        torch.utils.deterministic.fill_uninitialized_memory = True


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
    if os.environ.get("MTBLX_BOUNDS_CHECK") and "mtblx" in sys.modules:
        _bounds_check(request)


_bounds_seen = [0]


def _bounds_check(request):
    """the bounds-checked diagnostic library (oxidized-mtbl_amd/csrc/bounds.h, MTBLX_LIB pointing
    at build/libmtblx_bounds.so): fail the test whose launches touched memory outside their
    argument allocations, or faulted"""
    import ctypes as C
    import mtblx
    lib = mtblx.lib()
    fn = getattr(lib, "mtblx_bounds_report", None)
    if fn is None:
        return
    fn.restype = C.c_longlong
    fn.argtypes = [C.c_char_p, C.c_size_t]
    buf = C.create_string_buffer(512)
    n = int(fn(buf, 512))
    assert n >= 0, "MTBLX_BOUNDS_CHECK is set but the loaded library is not the bounds-checked build"
    if n != _bounds_seen[0]:
        _bounds_seen[0] = n
        pytest.fail(f"bounds-checked build: {n & 0xFFFFFFFF} out-of-allocation accesses, {n >> 32} faults "
                    f"so far; first: {buf.value.decode()}")
