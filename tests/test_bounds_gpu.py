"""The bounds-checked diagnostic build itself (oxidized-mtbl_amd/csrc/bounds.h, Makefile target
`bounds`): runs only when the GPU suite runs on that build (MTBLX_BOUNDS_CHECK=1,
MTBLX_LIB=.../build/libmtblx_bounds.so, tools/rounds/gpu_r05.sh MODES=bounds).

Positive control: with MTBLX_BOUNDS_SELFTEST=1 the decode launch's first pointer (the block
bytes) is left out of the checker's table, so its reads must be reported -- a clean suite run
means something only if the checker demonstrably reports."""
import os
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def test_checker_reports_a_withheld_buffer(monkeypatch):
    if not os.environ.get("MTBLX_BOUNDS_CHECK"):
        pytest.skip("product build: the bounds checker is a diagnostic build")
    import ctypes as C

    import torch
    import mtblx
    from mtblx import codec, synth
    lib = mtblx.lib()
    fn = lib.mtblx_bounds_report
    fn.restype = C.c_longlong
    fn.argtypes = [C.c_char_p, C.c_size_t]
    buf = C.create_string_buffer(512)
    before = int(fn(buf, 512))
    assert before >= 0
    data, off, ln = synth.cfg2_file(64)
    batch = codec.DeviceBatch.from_host(data, off, ln)
    monkeypatch.setenv("MTBLX_BOUNDS_SELFTEST", "1")
    codec.decode_blocks(batch)
    torch.cuda.synchronize()
    monkeypatch.delenv("MTBLX_BOUNDS_SELFTEST")
    after = int(fn(buf, 512))
    assert (after & 0xFFFFFFFF) > (before & 0xFFFFFFFF) and (after >> 32) == (before >> 32)
    assert b"k_decode_pipe" in buf.value or b"k_decode" in buf.value, buf.value
    # the reports above are this test's own: tell the per-test check (conftest) they were expected
    sys.modules["conftest"]._bounds_seen[0] = after
    # and without the self-test the same launch is clean
    codec.decode_blocks(batch)
    torch.cuda.synchronize()
    assert int(fn(buf, 512)) == after
