"""Host block codecs for every CompressionType (src/compression.rs:57-81; SURVEY.md §2 marks
compression host-only): None, Snappy (in-repo), Zlib (system zlib), Zstd (libzstd.so.1 at run
time), Lz4 / Lz4hc (the crate's Err "unsupported").

CPU: round trips, cross-checks against Python's own zlib, the oracle's decoders as the checker,
corrupt streams -> MTBLX_CODEC_CORRUPT (the crate's Error::Io), and whole files written with each
codec by the product Writer read back by the oracle Reader (src/reader.rs restated).
GPU: the device Reader, the end-to-end pipe and the C++ surface on Zlib / Zstd files vs the oracle.
"""
import ctypes as C
import os
import subprocess
import zlib

import numpy as np
import pytest

import corpus

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _lib():
    from mtblx import _lib
    return _lib, _lib.lib()


def _dec(comp, data: bytes):
    m, L = _lib()
    src = np.frombuffer(data or b"\0", np.uint8)
    out = m.u8p()
    n = C.c_uint64(0)
    rc = L.mtblx_decompress(comp, src.ctypes.data, len(data), C.byref(out), C.byref(n))
    if rc != 0:
        return rc, None
    b = C.string_at(out, n.value)
    L.mtblx_free(out)
    return 0, b


def _enc(comp, data: bytes, level=0):
    m, L = _lib()
    src = np.frombuffer(data or b"\0", np.uint8)
    out = m.u8p()
    n = C.c_uint64(0)
    assert L.mtblx_compress(comp, level, src.ctypes.data, len(data), C.byref(out), C.byref(n)) == 0
    b = C.string_at(out, n.value)
    L.mtblx_free(out)
    return b


def _samples():
    rng = np.random.default_rng(5)
    return [b"", b"x", rng.integers(0, 256, 5000, dtype=np.uint8).tobytes(), b"abcd" * 20000,
            bytes(rng.integers(0, 4, 70000, dtype=np.uint8))]


def _zstd_ok():
    return _lib()[1].mtblx_codec_available(5) == 1


@pytest.mark.parametrize("comp", [0, 1, 2, 5])
def test_round_trip(comp):
    if comp == 5 and not _zstd_ok():
        pytest.skip("libzstd.so.1 not on this host")
    for d in _samples():
        for lvl in (0, 1, 6):
            rc, back = _dec(comp, _enc(comp, d, lvl))
            assert rc == 0 and back == d


def test_zlib_matches_python_zlib():
    for d in _samples():
        for lvl in (0, 6, 9):
            assert _dec(2, zlib.compress(d, lvl)) == (0, d)        # the format flate2 reads
            assert zlib.decompress(_enc(2, d, lvl)) == d              # the format flate2 writes
    # bytes after the end of the stream are never read (ZlibDecoder stops at the stream end)
    assert _dec(2, zlib.compress(b"hello") + b"trailing") == (0, b"hello")


def test_corrupt_and_unsupported(oracle):
    m, _ = _lib()
    z = zlib.compress(b"hello world" * 100)
    assert _dec(2, z[: len(z) // 2])[0] == m.CODEC_CORRUPT       # input ends inside the stream
    assert _dec(2, b"")[0] == m.CODEC_CORRUPT
    assert _dec(2, b"\x00\x01\x02\x03")[0] == m.CODEC_CORRUPT
    for c in (3, 4, 9):                                          # Lz4 / Lz4hc: Err "unsupported"
        assert _dec(c, b"abc")[0] == m.CODEC_UNSUPPORTED
    if _zstd_ok():
        f = _enc(5, b"zstd frame " * 1000, 3)
        assert _dec(5, f[:-3])[0] == m.CODEC_CORRUPT              # cut inside the frame
        assert _dec(5, f + f) == (0, b"zstd frame " * 2000)       # every frame until the input ends
        assert _dec(5, b"") == (0, b"")
        assert _dec(5, b"\x01\x02\x03\x04\x05")[0] == m.CODEC_CORRUPT


@pytest.mark.parametrize("comp", [2, 5])
def test_files_read_by_oracle(oracle, comp):
    """the product Writer with Zlib / Zstd data blocks; the oracle Reader (with its own zlib /
    libzstd decoders) yields exactly the records, and the footer names the codec"""
    if comp == 5 and not _zstd_ok():
        pytest.skip("libzstd.so.1 not on this host")
    from mtblx.writer import Writer
    rng = np.random.default_rng(comp)
    recs = corpus.random_records(rng, 2500, 0, 40, 0, 200)
    for level in (0, 3):
        w = Writer(4096, 16, comp, level)
        for k, v in recs:
            w.insert(k, v)
        f = w.into_inner()
        s = oracle.file_scan(f, "iter")
        assert s["end"] == 0 and s["records"] == recs
        assert int.from_bytes(f[-512 + 16: -512 + 24], "little") == comp


def test_batch_decompress_layout():
    m, L = _lib()
    blocks = [zlib.compress(d) for d in _samples()] + [b"\x00bad"]
    file = b"".join(blocks)
    off = np.cumsum([0] + [len(b) for b in blocks[:-1]]).astype(np.uint64)
    ln = np.array([len(b) for b in blocks], np.uint32)
    n = len(blocks)
    dst = m.u8p()
    doff = np.zeros(n, np.uint64)
    dlen = np.zeros(n, np.uint64)
    st = np.zeros(n, np.int32)
    fa = np.frombuffer(file, np.uint8)
    bad = L.mtblx_decompress_blocks(2, fa.ctypes.data, off.ctypes.data, ln.ctypes.data, n, 4, C.byref(dst),
                                    doff.ctypes.data, dlen.ctypes.data, st.ctypes.data)
    assert bad == 1 and st.tolist() == [0] * (n - 1) + [m.CODEC_CORRUPT]
    for i, d in enumerate(_samples()):
        assert doff[i] % 16 == 0 and C.string_at(C.addressof(dst.contents) + int(doff[i]), int(dlen[i])) == d
    assert dlen[-1] == 0
    L.mtblx_free(dst)


# ------------------------------------------------------------------ GPU
def _write(recs, comp, bs=4096):
    from mtblx.writer import Writer
    w = Writer(bs, 16, comp, 1)
    for k, v in recs:
        w.insert(k, v)
    data = w.into_inner()
    return data, w.block_dir


@pytest.mark.gpu
@pytest.mark.parametrize("comp", [2, 5])
def test_device_reader_and_pipe(oracle, comp, tmp_path):
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    if comp == 5 and not _zstd_ok():
        pytest.skip("libzstd.so.1 not on this host")
    from mtblx import pipe, reader
    rng = np.random.default_rng(10 + comp)
    recs = corpus.random_records(rng, 6000, 0, 40, 0, 300)
    data, (off, ln) = _write(recs, comp)
    exp = oracle.file_scan(data, "iter")
    s = reader.Reader(data).iter()
    assert s.end == exp["end"] == 0 and s.records() == exp["records"] == recs
    assert reader.Reader(data).get(recs[1234][0]) == recs[1234][1]
    # a corrupted stored block: checksum off -> the block fails to decompress -> Err(Io) at next
    d2 = bytearray(data)
    d2[int(off[3]) + 5] ^= 0xFF
    e2 = oracle.file_scan(bytes(d2), "iter", verify=False)
    s2 = reader.ReaderBuilder().verify_checksums(False).read(bytes(d2)).iter()
    assert (s2.end, s2.err) == (e2["end"], e2["err"]) and s2.records() == e2["records"]
    # end-to-end pipe: host file in, host slices out
    nrec = sum(1 for _ in recs)
    kb = sum(len(k) for k, _ in recs)
    vb = sum(len(v) for _, v in recs)
    ho = pipe.HostOutputs(off.size, nrec, kb, vb)
    pipe.HostPipe(chunk_bytes=1 << 20).decode(np.frombuffer(data, np.uint8), off, ln, ho, compression=comp)
    assert tuple(int(x) for x in ho.totals) == (nrec, kb, vb, 0)
    got = [r for b in range(off.size) for r in ho.records(b)]
    assert got == recs
    # C++ surface: examples/dump.rs over the file
    dump = os.path.join(ROOT, "oxidized-mtbl_amd", "build", "dump")
    if os.path.exists(dump):
        p = tmp_path / "f.mtbl"
        p.write_bytes(data)
        r = subprocess.run([dump, str(p)], capture_output=True, timeout=120)
        assert r.returncode == 0
        assert r.stdout == b"".join(b'"' + k + b'" "' + v + b'"\n' for k, v in recs)


@pytest.mark.parametrize("comp", [3, 4])
def test_writer_lz4_err_semantics(oracle, comp):
    """WriterBuilder with Lz4 / Lz4hc (src/writer.rs:112-237, src/compression.rs:70-81): inserts
    succeed until the first data-block flush, whose compress() returns Err "unsupported ...":
    that insert returns the Err and its record is not added.  The data BlockBuilder's buffer was
    moved out by finish() and never reset, so the next insert panics on `assert!(!finished)`
    (src/block_builder.rs:51), while into_inner still succeeds -- the flush sees an empty block --
    and writes the index and a footer whose counts include the lost block's records.  An Lz4
    writer that never flushes a data block writes an ordinary empty file."""
    from mtblx.writer import Writer, WriterIoError, WriterPanic
    f = Writer(1024, 16, comp).into_inner()
    s = oracle.file_scan(f, "iter")
    assert s["end"] == 0 and s["records"] == []
    assert int.from_bytes(f[-512 + 16: -512 + 24], "little") == comp

    recs = [(b"k%04d" % i, b"v" * 60) for i in range(40)]
    w = Writer(1024, 16, comp)
    n = 0
    with pytest.raises(WriterIoError, match="unsupported Lz4"):
        for k, v in recs:
            w.insert(k, v)
            n += 1
    assert 0 < n < len(recs)                       # the Err came from the first flush
    with pytest.raises(WriterPanic):
        w.insert(recs[n + 1][0], recs[n + 1][1])   # assert!(!self.finished) in BlockBuilder::add
    w2 = Writer(1024, 16, comp)
    for k, v in recs[:n]:
        w2.insert(k, v)
    with pytest.raises(WriterIoError):
        w2.insert(*recs[n])
    out = w2.into_inner()                          # flush: the data block is empty -> Ok
    meta = [int.from_bytes(out[-512 + 8 * i: -512 + 8 * i + 8], "little") for i in range(9)]
    assert meta[2] == comp and meta[3] == n and meta[4] == 0    # count_entries n, no data block
    s = oracle.file_scan(out, "iter")
    assert s["records"] == []
