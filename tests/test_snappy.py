"""Host snappy codec (CompressionType::Snappy, src/compression.rs:116-130) and snappy files.

The product codec (csrc/snappy_host.cpp) is checked against the oracle's independent
byte-at-a-time restatement (oracle/mtbl_oracle.c) and, where this image has it, against
libsnappy 1.1.8 (/opt/conda/lib, not shipped by the reference: `snap` itself is a Rust crate
absent from /root/reference, so its published format is the pin).  Compressed BYTES are
parity-unpinned; only round trips and decoded bytes are compared.
"""
import ctypes as C
import os

import numpy as np
import pytest

import corpus


def _libsnappy():
    for p in ("/opt/conda/lib/libsnappy.so.1", "/opt/conda/lib/libsnappy.so"):
        if os.path.exists(p):
            try:
                L = C.CDLL(p)
            except OSError:
                continue
            L.snappy_compress.argtypes = [C.c_char_p, C.c_size_t, C.c_char_p, C.POINTER(C.c_size_t)]
            L.snappy_uncompress.argtypes = [C.c_char_p, C.c_size_t, C.c_char_p, C.POINTER(C.c_size_t)]
            L.snappy_max_compressed_length.argtypes = [C.c_size_t]
            L.snappy_max_compressed_length.restype = C.c_size_t
            L.snappy_uncompressed_length.argtypes = [C.c_char_p, C.c_size_t, C.POINTER(C.c_size_t)]
            return L
    return None


def _inputs():
    rng = np.random.default_rng(7)
    out = [b"", b"a", b"ab" * 3, bytes(range(256)), b"\0" * 100_000, b"abcd" * 40_000]
    out += [rng.integers(0, 256, int(n), dtype=np.uint8).tobytes() for n in (59, 60, 61, 255, 256, 65535, 65536,
                                                                            65537, 200_000)]
    # compressible structured data: mtbl blocks
    from mtblx import synth
    data, off, ln = synth.cfg2_file(8)
    out += [bytes(data[int(o): int(o) + int(n)]) for o, n in zip(off, ln)]
    recs = corpus.random_records(rng, 400, 0, 60, 0, 30)
    out.append(b"".join(k + v for k, v in recs))
    return out


def test_product_roundtrip_and_oracle_agree(oracle):
    from mtblx import pipe
    for x in _inputs():
        z = pipe.snappy_compress(x)
        assert pipe.snappy_decompress(z) == x
        assert oracle.snappy_decompress(z) == x


def test_libsnappy_cross_check(oracle):
    from mtblx import pipe
    L = _libsnappy()
    if L is None:
        pytest.skip("libsnappy not in this image")
    for x in _inputs():
        # libsnappy -> product + oracle
        cap = L.snappy_max_compressed_length(len(x))
        buf = C.create_string_buffer(cap)
        n = C.c_size_t(cap)
        assert L.snappy_compress(x, len(x), buf, C.byref(n)) == 0
        z = buf.raw[: n.value]
        assert pipe.snappy_decompress(z) == x
        assert oracle.snappy_decompress(z) == x
        # product -> libsnappy
        z2 = pipe.snappy_compress(x)
        out = C.create_string_buffer(max(len(x), 1))
        m = C.c_size_t(max(len(x), 1))
        assert L.snappy_uncompress(z2, len(z2), out, C.byref(m)) == 0
        assert out.raw[: m.value] == x


def test_corrupt_streams_agree(oracle):
    """mutated streams: product and oracle agree on error vs bytes (Err(Io) where snap errors)"""
    from mtblx import pipe
    rng = np.random.default_rng(11)
    base = [pipe.snappy_compress(x) for x in _inputs() if len(x) < 70_000]
    errors = 0
    for i in range(3000):
        z = bytearray(base[i % len(base)])
        if not z:
            continue
        k = int(rng.integers(0, 4))
        if k == 0:
            z[int(rng.integers(0, len(z)))] ^= 1 << int(rng.integers(0, 8))
        elif k == 1:
            z = z[: int(rng.integers(0, len(z)))]
        elif k == 2:
            z[0] = int(rng.integers(0, 256))
        else:
            j = int(rng.integers(0, len(z)))
            z[j] = int(rng.integers(0, 256))
        a = pipe.snappy_decompress(bytes(z))
        b = oracle.snappy_decompress(bytes(z))
        assert a == b, i
        errors += a is None
    assert errors > 100


def test_snappy_file_reads_back(oracle):
    """Writer with CompressionType::Snappy: the oracle Reader (snappy restated) yields exactly
    the records, the footer says Snappy, and every data block decompresses to the block the
    None-compressed file holds at the same position (the flush rule uses uncompressed sizes,
    src/writer.rs:125-130, so both files cut blocks identically)."""
    from mtblx import pipe, synth
    from mtblx.writer import Writer
    rng = np.random.default_rng(5)
    recs = corpus.random_records(rng, 3000, 1, 40, 0, 120)
    files = {}
    for comp in (0, 1):
        w = Writer(4096, 16, comp)
        for k, v in recs:
            w.insert(k, v)
        files[comp] = (w.into_inner(), w.block_dir)
    (d0, (o0, l0)), (d1, (o1, l1)) = files[0], files[1]
    exp = oracle.file_scan(d1, "iter")
    assert exp["end"] == 0 and exp["records"] == recs
    assert exp["meta"][2] == 1 and exp["meta"][3] == len(recs)
    assert o0.size == o1.size
    assert sum(int(x) for x in l1) < sum(int(x) for x in l0)
    for a, n, b, m in zip(o0, l0, o1, l1):
        assert pipe.snappy_decompress(d1[int(b): int(b) + int(m)]) == d0[int(a): int(a) + int(n)]
    # cfg1 file with snappy
    w = Writer(4096, 16, 1)
    for k, v in synth.cfg1_records():
        w.insert(k, v)
    assert len(oracle.file_scan(w.into_inner(), "iter")["records"]) == 10_000


def test_snappy_file_corrupt_block_is_io_error(oracle):
    """a data block whose stored bytes are valid for the CRC but not valid snappy -> Err(Io)"""
    from mtblx.writer import Writer
    rng = np.random.default_rng(6)
    recs = corpus.random_records(rng, 800, 1, 20, 0, 50)
    w = Writer(1024, 16, 1)
    for k, v in recs:
        w.insert(k, v)
    d = bytearray(w.into_inner())
    off, ln = w.block_dir
    b = 2
    d[int(off[b])] = 0xFF   # preamble: unterminated varint byte -> still varint, wrong length
    d[int(off[b]) + 1] = 0xFF
    d[int(off[b]) + 2] = 0xFF
    r = oracle.file_scan(bytes(d), "iter", verify=False)
    assert r["end"] == 2 and r["err"] == "Io"   # END_ERR_NEXT
