"""Device snappy raw decompression (f4, include/mtblx.h mtblx_snappy_dir /
mtblx_snappy_decompress_dev) against the oracle's independent byte-at-a-time restatement
(oracle/mtbl_oracle.c oracle_snappy_decompress; Reader::block -> src/compression.rs:116-119).

Streams come from the product compressor and, where this image has it, libsnappy 1.1.8 (a
different encoder: different element mixes).  Compressed bytes are parity-unpinned (SURVEY.md
§8c); decoded bytes and the error/ok verdict per block are compared.  Shapes cover both kernel
variants (<= 4.5 KiB outputs: Small; larger: Large, with outputs above 65 KiB assembled in HBM),
overlapping copies (period 1..4), literals longer than a staging window, empty streams and
mutated streams.
"""
import numpy as np
import pytest

import corpus
from test_snappy import _inputs, _libsnappy

pytestmark = pytest.mark.gpu


@pytest.fixture(params=["auto", "lanes", "two", "waves"], autouse=True)
def snappy_kernel(request, monkeypatch):
    """every test under the default routing, with every block on k_snappy_lanes (one lane per
    block, output streamed to HBM) -- auto sends blocks there only in large batches -- and with
    the blocks expanding > 2x on the two-pass kernels (k_snappy_parse + k_snappy_exec) whatever
    the batch size"""
    if request.param in ("lanes", "two", "waves"):
        monkeypatch.setenv("MTBLX_SNAPPY_KERNEL", request.param)
    else:
        monkeypatch.delenv("MTBLX_SNAPPY_KERNEL", raising=False)
    return request.param


def _dev():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from mtblx import codec
    return codec


def _streams(xs, lib=None):
    from mtblx import pipe
    out = []
    for x in xs:
        out.append(pipe.snappy_compress(x))
        if lib is not None:
            import ctypes as C
            cap = lib.snappy_max_compressed_length(len(x))
            buf = C.create_string_buffer(cap)
            n = C.c_size_t(cap)
            assert lib.snappy_compress(x, len(x), buf, C.byref(n)) == 0
            out.append(buf.raw[: n.value])
    return out


def _device(codec, streams, rng, lead=0):
    data, off, ln = corpus.pack(streams, rng=rng, lead=lead)
    batch = codec.SnappyBatch.from_host(data, off, ln)
    dec, st = codec.snappy_decompress(batch)
    import torch
    torch.cuda.synchronize()
    host = dec.data.cpu().numpy()
    o = dec.blk_off.cpu().numpy().view(np.uint64)
    n = dec.blk_len.cpu().numpy().view(np.uint32)
    got = [bytes(host[int(a): int(a) + int(b)]) for a, b in zip(o, n)]
    return got, st.cpu().numpy(), o


def _check(oracle, streams, got, st):
    for i, z in enumerate(streams):
        exp = oracle.snappy_decompress(z)
        if exp is None:
            assert st[i] == 1, i
        else:
            assert st[i] == 0, (i, st[i])
            assert got[i] == exp, i


def _compressible(rng):
    xs = [b"", b"x", b"ab" * 2000, b"\0" * 4500, bytes(range(256)) * 17, b"abc" * 1500, b"abcd" * 16_000]
    xs += [b"".join(rng.choice([b"alpha", b"beta", b"gamma", b"delta"], 2000).tolist())]
    from mtblx import synth
    xs += [b"".join(v for _, v in synth.cfg1_records(400))]
    recs = corpus.random_records(rng, 300, 0, 40, 0, 20)
    xs.append(b"".join(k + v for k, v in recs))
    return xs


def test_small_blocks_vs_oracle(oracle):
    """every output <= 4.5 KiB: the Small variant (16 waves per CU, LDS output)"""
    codec = _dev()
    rng = np.random.default_rng(1)
    from mtblx import synth
    data, off, ln = synth.cfg2_file(300)
    xs = [bytes(data[int(a): int(a) + int(n)]) for a, n in zip(off, ln)]
    xs += [x for x in _compressible(rng) if len(x) <= 4608]
    xs += [rng.integers(0, 256, int(n), dtype=np.uint8).tobytes() for n in (1, 2, 3, 15, 16, 17, 59, 60, 61, 4608)]
    streams = _streams(xs, _libsnappy())
    got, st, o = _device(codec, streams, rng, lead=3)
    _check(oracle, streams, got, st)
    assert (o % 16 == 0).all()


def _varint(n):
    out = bytearray()
    while True:
        b = n & 0x7F
        n >>= 7
        out.append(b | (0x80 if n else 0))
        if not n:
            return bytes(out)


def _lit4(b):   # a literal with a 4-byte length field (the longest legal header)
    return bytes([63 << 2]) + (len(b) - 1).to_bytes(4, "little") + b


def _copy4(length, off):   # a copy with a 4-byte offset, 1..64 bytes
    return bytes([((length - 1) << 2) | 3]) + off.to_bytes(4, "little")


def _copy2(length, off):
    return bytes([((length - 1) << 2) | 2]) + off.to_bytes(2, "little")


def test_small_blocks_wasteful_encodings_vs_oracle(oracle):
    """valid streams whose encodings are far longer than their output (<= 4.5 KiB, the
    four-blocks-per-wave kernel): tag bytes and literal bytes past its 4752-byte LDS window are
    read from HBM; a literal straddling the window end; long runs of 1-byte copies"""
    codec = _dev()
    rng = np.random.default_rng(5)
    streams = []
    out = rng.integers(0, 256, 1000, dtype=np.uint8).tobytes()
    streams.append(_varint(1000) + b"".join(_lit4(out[i: i + 1]) for i in range(1000)))   # 6 B per byte
    tail = rng.integers(0, 256, 1500, dtype=np.uint8).tobytes()
    streams.append(_varint(3001 + 1500) + bytes([0]) + b"A" + b"".join(_copy4(1, 1) for _ in range(3000)) + _lit4(tail))
    # a literal starting inside the window and ending past it
    pre = b"".join(_copy2(1, 1) for _ in range(1500))   # 3 B per output byte
    mid = rng.integers(0, 256, 1200, dtype=np.uint8).tobytes()
    streams.append(_varint(1 + 1500 + 1200) + bytes([0]) + b"z" + pre + _lit4(mid))
    # random element mix, some copies reaching back the whole block
    for seed in range(6):
        r = np.random.default_rng(100 + seed)
        body, produced, parts = bytearray(), 0, []
        first = r.integers(0, 256, 8, dtype=np.uint8).tobytes()
        body += _lit4(first)
        parts.append(first)
        produced = 8
        while produced < 4000:
            k = int(r.integers(0, 3))
            if k == 0:
                b = r.integers(0, 256, int(r.integers(1, 90)), dtype=np.uint8).tobytes()
                body += _lit4(b)
                parts.append(b)
                produced += len(b)
            else:
                ln = int(r.integers(1, 65))
                off = int(r.integers(1, produced + 1))
                body += _copy4(ln, off) if k == 1 else _copy2(ln, min(off, 65535))
                o = min(off, 65535) if k == 2 else off
                cur = b"".join(parts)
                piece = bytearray()
                for i in range(ln):
                    piece.append((cur + bytes(piece))[len(cur) - o + i])
                parts.append(bytes(piece))
                produced += ln
        streams.append(_varint(produced) + bytes(body))
    # output that catches up with its unread stored bytes: a copy-heavy head (3009 bytes from
    # ~144 stored bytes) then 1500 one-byte literals with 1-byte tags (2 stored bytes each) --
    # the shared-buffer kernel must hand this block to the deferred pass
    lits = rng.integers(0, 256, 1500, dtype=np.uint8).tobytes()
    streams.append(_varint(1 + 47 * 64 + 1500) + bytes([0]) + b"A" + _copy2(64, 1) * 47 +
                   b"".join(bytes([0]) + lits[i: i + 1] for i in range(1500)))
    assert all(len(z) > 4752 for z in streams[:3])
    from mtblx import pipe
    streams += [pipe.snappy_compress(bytes(rng.integers(0, 256, 3000, dtype=np.uint8)))] * 5
    got, st, _ = _device(codec, streams, rng, lead=5)
    _check(oracle, streams, got, st)
    assert (st == 0).all()


def test_mixed_and_large_blocks_vs_oracle(oracle):
    """outputs up to 200 KB: the Large variant, in-HBM assembly above 65 KiB, long literals
    crossing staging windows, overlapping copies"""
    codec = _dev()
    rng = np.random.default_rng(2)
    xs = _inputs() + _compressible(rng)
    xs += [rng.integers(0, 256, 70_000, dtype=np.uint8).tobytes(), b"q" * 66_000, b"xy" * 40_000]
    streams = _streams(xs, _libsnappy())
    got, st, _ = _device(codec, streams, rng, lead=1)
    _check(oracle, streams, got, st)


def test_corrupt_streams_vs_oracle(oracle):
    """mutated streams (bit flips, truncations, preamble rewrites, random bytes): the device
    flags exactly the streams the oracle rejects and decodes the rest identically"""
    codec = _dev()
    from mtblx import pipe
    rng = np.random.default_rng(11)
    base = [pipe.snappy_compress(x) for x in _inputs() + _compressible(rng) if len(x) < 70_000]
    streams = []
    for i in range(3000):
        z = bytearray(base[i % len(base)])
        if not z:
            streams.append(bytes(z))
            continue
        k = int(rng.integers(0, 4))
        if k == 0:
            z[int(rng.integers(0, len(z)))] ^= 1 << int(rng.integers(0, 8))
        elif k == 1:
            z = z[: int(rng.integers(0, len(z)))]
        elif k == 2:
            z[0] = int(rng.integers(0, 256))
        else:
            z[int(rng.integers(0, len(z)))] = int(rng.integers(0, 256))
        streams.append(bytes(z))
    got, st, _ = _device(codec, streams, rng)
    _check(oracle, streams, got, st)
    assert (st == 1).sum() > 300 and (st == 0).sum() > 300


def test_too_small_capacity():
    """a block whose preamble length exceeds its dst_len capacity -> MTBLX_SNAPPY_TOO_SMALL"""
    codec = _dev()
    import torch
    from mtblx import pipe
    xs = [b"a" * 100, b"b" * 300, b"c" * 50]
    zs = [pipe.snappy_compress(x) for x in xs]
    data, off, ln = corpus.pack(zs)
    batch = codec.SnappyBatch.from_host(data, off, ln)
    lay = codec.SnappyLayout(3)
    codec.snappy_dir(batch, lay)
    torch.cuda.synchronize()
    assert lay.dst_len.cpu().tolist() == [100, 300, 50]
    assert lay.dst_off.cpu().tolist() == [0, 112, 416]
    assert lay.totals.cpu().tolist() == [416 + 64, 300, 0]
    lay.dst_len[1] = 299
    dst = torch.zeros(1024, dtype=torch.uint8, device="cuda")
    st = torch.full((3,), -1, dtype=torch.int32, device="cuda")
    dl = torch.full((3,), -1, dtype=torch.int32, device="cuda")
    codec.snappy_decompress_into(batch, lay, dst, st, dl, 300)
    torch.cuda.synchronize()
    assert st.cpu().tolist() == [0, 2, 0] and dl.cpu().tolist() == [100, 0, 50]
    h = dst.cpu().numpy().tobytes()
    assert h[:100] == xs[0] and h[416:466] == xs[2]


def test_snappy_file_device_decompress_then_decode(oracle):
    """a CompressionType::Snappy file: device decompression feeds the device decode directly
    ({dst, dst_off, dec_len} is the decode batch); records == the None file's decode by the
    oracle, with one corrupted block reported CORRUPT and decoded as empty (INVALID_BLOCK)"""
    codec = _dev()
    from mtblx.writer import Writer
    rng = np.random.default_rng(9)
    recs = corpus.random_records(rng, 6000, 1, 40, 0, 120)
    files = {}
    for comp in (0, 1):
        w = Writer(4096, 16, comp)
        for k, v in recs:
            w.insert(k, v)
        files[comp] = (np.frombuffer(w.into_inner(), np.uint8).copy(), *w.block_dir)
    d0, o0, l0 = files[0]
    d1, o1, l1 = files[1]
    exp = oracle.decode_blocks(d0, o0, l0)
    d1 = d1.copy()
    d1[int(o1[7])] ^= 0x01   # preamble length off by one -> snap error
    batch = codec.SnappyBatch.from_host(d1, o1, l1)
    dec, st = codec.snappy_decompress(batch)
    out = codec.decode_blocks(dec)
    import torch
    torch.cuda.synchronize()
    st = st.cpu().numpy()
    assert st[7] == 1 and (np.delete(st, 7) == 0).all()
    h = out.to_host()
    for b in range(o0.size):
        if b == 7:
            assert h.status[b] == 1 and h.nrec[b] == 0
        else:
            assert h.status[b] == 0 and h.records(b) == exp.records(b)


def test_auto_routing_large_batch(oracle, snappy_kernel):
    """a batch of 60 000 blocks (>= the 49 152 from which auto routes blocks expanding > 2x to
    k_snappy_lanes): compressible, random and corrupt streams mixed, so the quad kernel, the
    lanes kernel (blocks the quads mark) and the deferred pass all run in one call; under
    "two" the marked blocks take the parse / execute kernels, whose workgroups then loop over
    several quads each, and under "lanes" every block is one lane's"""
    codec = _dev()
    from mtblx import pipe, synth
    rng = np.random.default_rng(21)
    distinct = [pipe.snappy_compress(x) for x in _compressible(rng) if len(x) <= 4608]
    recs = list(synth.cfg1_records(4000))
    for i in range(0, 4000, 50):   # cfg1-style blocks of 50 records (<= 4500 bytes: the quad path)
        distinct.append(pipe.snappy_compress(b"".join(k + v for k, v in recs[i: i + 50])))
    distinct += [pipe.snappy_compress(rng.integers(0, 256, int(n), dtype=np.uint8).tobytes()) for n in (100, 3000, 4000)]
    bad = bytearray(distinct[-5])
    bad[len(bad) // 2] ^= 0x40
    distinct.append(bytes(bad))
    expect = [oracle.snappy_decompress(z) for z in distinct]
    pick = rng.integers(0, len(distinct), 60_000)
    streams = [distinct[int(i)] for i in pick]
    assert max(len(e) for e in expect if e is not None) <= 4608
    got, st, _ = _device(codec, streams, rng)
    for j, i in enumerate(pick):
        e = expect[int(i)]
        if e is None:
            assert st[j] == 1, j
        else:
            assert st[j] == 0 and got[j] == e, j
    ratios = [len(e) / max(len(z), 1) for z, e in zip(distinct, expect) if e is not None]
    assert max(ratios) > 2 and min(ratios) < 2   # both kernels took blocks


def test_long_block_beside_short_ones(oracle, snappy_kernel):
    """one lane decoding a multi-MB block in the same wave as short blocks.  Each
    decoding lane now publishes its end as soon as its own block is done, so the short blocks'
    writer lanes finish their last partial chunk at once instead of idling until the whole wave
    is done (past their 2 s guard, which left the tail unwritten under status OK)."""
    codec = _dev()
    rng = np.random.default_rng(77)
    phrases = [bytes(rng.integers(0, 256, int(n), dtype=np.uint8)) for n in (5, 9, 17, 33, 300)]
    big = b"".join(phrases[int(i)] for i in rng.integers(0, 5, 90_000))   # ~6 MB, copies of all offsets
    xs = [bytes(rng.integers(0, 256, int(n), dtype=np.uint8)) + b"q" * int(n) for n in rng.integers(1, 3000, 40)]
    xs.insert(17, big)
    streams = _streams(xs)
    got, st, _ = _device(codec, streams, rng)
    _check(oracle, streams, got, st)
    assert (st == 0).all()
