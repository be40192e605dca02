"""FormatV1 files on the CPU: the hand-derived V1 known-answer files, the oracle's V1 branch, and
the product's host-side footer / framing (no GPU needed).

The reference reads V1 (/root/reference/src/metadata.rs:29-33: magic 0x77846676;
src/reader.rs:54-56 index and :146-148 data blocks: u32 LE content length instead of varint64)
but never writes it (src/writer.rs:215), and holds no V1 file.  The pins are therefore:
  - tests/golden/one_key_v1.mtbl / empty_v1.mtbl, assembled in tests/golden/make_golden.py from
    hand-derived pieces (kat.json one_key_v1 / empty_v1, sha256 stated) and equal to what
    tests/corpus.py:to_v1 makes of the V2 goldens;
  - V1 copies of Writer output made by corpus.to_v1: the same stored block bytes re-framed, so
    every reading mode must yield exactly what the V2 original yields.
"""
import ctypes as C
import hashlib
import json
import os

import numpy as np
import pytest

import corpus

HERE = os.path.dirname(os.path.abspath(__file__))
END_NONE, END_ERR_OPEN, END_ERR_NEXT, END_PANIC = 0, 1, 2, 3   # oracle_file_scan end codes
GOLD = os.path.join(HERE, "golden")


def _kat():
    return json.load(open(os.path.join(GOLD, "kat.json")))


def test_v1_golden_files(oracle):
    kat = _kat()
    for name, v2 in (("one_key_v1", "one_key.mtbl"), ("empty_v1", "empty.mtbl")):
        k = kat[name]
        b = open(os.path.join(GOLD, name + ".mtbl"), "rb").read()
        assert len(b) == k["file_len"]
        if "sha256" in k:
            assert hashlib.sha256(b).hexdigest() == k["sha256"]
        # the hand-derived pieces, in order: data frame, index frame, footer, magic at 508
        frames = bytes.fromhex(k.get("data_frame", "") + k["index_frame"])
        assert b[: len(frames)] == frames
        assert [int.from_bytes(b[len(frames) + 8 * i: len(frames) + 8 * i + 8], "little") for i in range(9)] == \
            k["metadata"]
        assert b[-4:] == bytes.fromhex(k["magic"]) == corpus.MAGIC_V1.to_bytes(4, "little")
        assert corpus.to_v1(open(os.path.join(GOLD, v2), "rb").read()) == b
        r = oracle.file_scan(b)
        assert (r["version"], r["end"], r["meta"]) == (0, 0, k["metadata"])
        assert r["records"] == [(x.encode(), y.encode()) for x, y in k["records"]]
    one = open(os.path.join(GOLD, "one_key_v1.mtbl"), "rb").read()
    assert oracle.file_scan(one, "get", key=b"hello")["records"] == [(b"hello", b"I'm the one")]
    assert oracle.file_scan(one, "get", key=b"hellp")["records"] == []


def _files(oracle, rng):
    """oracle Writer output (CompressionType::None) and product Writer output for the codecs
    (the oracle writes None only; the product Writer is byte-identical to it on None)"""
    from mtblx.writer import Writer
    out = []
    for bs, iv, n, comp in ((1024, 1, 300, 0), (4096, 16, 1500, 0), (512, 3, 400, 1), (2048, 7, 600, 2),
                            (8192, 16, 2000, 5), (65536, 16, 3000, 0)):
        recs = corpus.random_records(rng, n, 0, 60, 0, 150)
        if comp == 0:
            out.append((oracle.write_file(recs, bs, iv, comp), recs))
        else:
            w = Writer(bs, iv, comp)
            for k, v in recs:
                w.insert(k, v)
            out.append((w.into_inner(), recs))
    out.append((oracle.write_file([], 4096, 16, 0), []))
    return out


def test_v1_copies_read_like_v2(oracle):
    """every reading mode of the oracle on a V1 copy == on the V2 original (same stored bytes)"""
    rng = np.random.default_rng(111)
    for v2, recs in _files(oracle, rng):
        v1 = corpus.to_v1(v2)
        a, b = oracle.file_scan(v2), oracle.file_scan(v1)
        assert b["version"] == 0 and a["version"] == 1
        assert (b["end"], b["records"]) == (a["end"], a["records"]) and len(b["records"]) == len(recs)
        assert b["end"] == END_NONE
        keys = [k for k, _ in recs] or [b"x"]
        for _ in range(6):
            k = keys[int(rng.integers(0, len(keys)))]
            for mode, k1, k2 in (("get", k, b""), ("from", k, b""), ("prefix", k[:2], b""), ("range", k, k + b"\xff")):
                x, y = oracle.file_scan(v2, mode, k1, k2), oracle.file_scan(v1, mode, k1, k2)
                assert (y["end"], y["records"]) == (x["end"], x["records"]), (mode, k1)
            ops = [3, ("seek", k), 5, ("seek", k[:1]), 2]
            x, y = oracle.iter_script(v2, "iter", b"", b"", ops), oracle.iter_script(v1, "iter", b"", b"", ops)
            assert (y["end"], y["records"], y["ops"]) == (x["end"], x["records"], x["ops"])


def test_v1_host_footer_and_framing(mtblx_lib, oracle):
    """mtblx_read_footer / mtblx_frame_block (csrc/host.cpp) on V1: version 0, u32 framing,
    the checksum assert, and a length past the end of the file (the reference's slice panics)"""
    import mtblx._lib as L
    b = open(os.path.join(GOLD, "one_key_v1.mtbl"), "rb").read()
    a = (C.c_uint8 * len(b)).from_buffer_copy(b)
    ft = L.Footer()
    assert mtblx_lib.mtblx_read_footer(a, len(b), C.byref(ft)) == 0
    assert list(ft.meta) == [35, 8192, 0, 1, 1, 35, 25, 5, 11] and ft.version == 0
    co, cl, pn = C.c_uint64(), C.c_uint64(), C.c_int()
    assert mtblx_lib.mtblx_frame_block(a, len(b), 0, 0, 1, C.byref(co), C.byref(cl), C.byref(pn)) == 0
    assert (co.value, cl.value, pn.value) == (8, 27, 0)                # data block: 4 + 4 framing bytes
    assert mtblx_lib.mtblx_frame_block(a, len(b), 0, 35, 1, C.byref(co), C.byref(cl), C.byref(pn)) == 0
    assert (co.value, cl.value, pn.value) == (43, 17, 0)               # the index block
    for patch, verify in (((0, 0x1c), 1), ((0, 0x1c), 0), ((3, 0x80), 1), ((3, 0x80), 0)):
        d = bytearray(b)
        d[patch[0]] = patch[1]        # 28 bytes (checksum / content mismatch) or 2 GiB past the end
        x = (C.c_uint8 * len(d)).from_buffer_copy(bytes(d))
        rc = mtblx_lib.mtblx_frame_block(x, len(d), 0, 0, verify, C.byref(co), C.byref(cl), C.byref(pn))
        past = patch[0] == 3
        assert pn.value == (1 if (past or verify) else 0), (patch, verify)
        if not pn.value:
            assert rc == 0 and (co.value, cl.value) == (8, 28)


@pytest.mark.parametrize("verify", [True, False])
def test_v1_corrupt_lengths_oracle(oracle, verify):
    """the oracle's V1 branch on corrupted u32 lengths: past the file end -> panic (slice
    assert, src/reader.rs:155); shorter -> a checksum panic when verifying, else the block scan
    of the truncated content; an index length past the end -> panic at open"""
    rng = np.random.default_rng(7)
    recs = corpus.random_records(rng, 800, 4, 30, 10, 80)
    v1 = corpus.to_v1(oracle.write_file(recs, 2048, 8, 0))
    frames = corpus.v1_frames(v1)
    base = oracle.file_scan(v1, verify=verify)
    assert base["end"] == 0 and len(base["records"]) == len(recs)
    off, n = frames[3]
    d = bytearray(v1)
    d[off: off + 4] = (len(v1) + 100).to_bytes(4, "little")
    assert oracle.file_scan(bytes(d), verify=verify)["end"] == END_PANIC
    d = bytearray(v1)
    d[off: off + 4] = (n - 9).to_bytes(4, "little")
    r = oracle.file_scan(bytes(d), verify=verify)
    assert r["end"] != END_NONE
    if verify:
        assert r["end"] == END_PANIC and len(r["records"]) < len(recs)
    io, ni = frames[-1]
    d = bytearray(v1)
    d[io: io + 4] = (1 << 31).to_bytes(4, "little")
    assert oracle.file_scan(bytes(d), verify=verify)["end"] == END_PANIC
