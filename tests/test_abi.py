"""The C-ABI library loads and exports every symbol include/*.h declares (no GPU calls)."""
import ctypes as C
import glob
import os
import re
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_functions():
    names = set()
    for h in glob.glob(os.path.join(ROOT, "include", "*.h")):
        src = open(h).read()
        src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
        for m in re.finditer(r"\b(mtblx_[a-z0-9_]+)\s*\(", src):
            names.add(m.group(1))
    return names


def test_headers_declare_functions():
    names = declared_functions()
    assert "mtblx_decode_blocks" in names and "mtblx_count_blocks" in names
    assert len(names) >= 15


def test_library_exports_all_declared(mtblx_lib):
    import mtblx
    out = subprocess.run(["nm", "-D", "--defined-only", mtblx.LIB_PATH], capture_output=True, text=True).stdout
    exported = {ln.split()[-1] for ln in out.splitlines() if " T " in ln}
    missing = declared_functions() - exported
    assert not missing, missing
    assert set(mtblx.EXPORTS) <= exported
    for n in declared_functions():
        assert getattr(mtblx_lib, n) is not None


def test_abi_version(mtblx_lib):
    assert mtblx_lib.mtblx_abi_version() == 3


def test_workspace_size_monotone(mtblx_lib):
    a = mtblx_lib.mtblx_decode_workspace_bytes(1000)
    b = mtblx_lib.mtblx_decode_workspace_bytes(100000)
    assert 0 < a < b


def test_decode_rejects_null_args(mtblx_lib):
    # argument checks happen before any device work
    from mtblx._lib import BlockBatch, Decoded
    b = BlockBatch(0, 0, 0, 0, 5, 0)
    o = Decoded()
    rc = mtblx_lib.mtblx_decode_blocks(C.byref(b), C.byref(o), None, 0, None)
    assert rc == -1


def test_footer_and_framing(mtblx_lib, oracle):
    import mtblx
    from mtblx._lib import Footer, u8p
    f = oracle.write_file([(b"hello", b"I'm the one")])
    a = (C.c_uint8 * len(f)).from_buffer_copy(f)
    ft = Footer()
    assert mtblx_lib.mtblx_read_footer(a, len(f), C.byref(ft)) == 0
    assert list(ft.meta) == [32, 8192, 0, 1, 1, 32, 22, 5, 11] and ft.version == 1
    co, cl, pn = C.c_uint64(), C.c_uint64(), C.c_int()
    assert mtblx_lib.mtblx_frame_block(a, len(f), 1, 0, 1, C.byref(co), C.byref(cl), C.byref(pn)) == 0
    assert (co.value, cl.value, pn.value) == (5, 27, 0)
    bad = bytearray(f)
    bad[10] ^= 1
    b2 = (C.c_uint8 * len(bad)).from_buffer_copy(bytes(bad))
    assert mtblx_lib.mtblx_frame_block(b2, len(bad), 1, 0, 1, C.byref(co), C.byref(cl), C.byref(pn)) != 0
    assert pn.value == 1
    del mtblx, u8p
