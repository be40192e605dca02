"""Blocks >= 4 GiB (Block::init's u64 restart array, src/block.rs:25-42,
restart_point's 4-byte stride on it, :95-104; BlockBuilder::finish switches to u64 restarts past
u32::MAX, src/block_builder.rs:85-97).  A ~4.3 GiB block written by the product Writer (block size
4 GiB: three small records, two ~2 GiB values, then a second, small block) read by the device
Reader -- the big block framed from its index entry, checksummed in 1 GiB pieces, decoded by the
emitting block seek -- against the oracle's restatement; Reader::get into it."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _file():
    from mtblx.writer import Writer
    vlen = (1 << 31) + 4099
    pat = np.tile(np.arange(256, dtype=np.uint8), vlen // 256 + 1)[:vlen]
    v1 = pat.tobytes()
    v2 = (pat * np.uint8(7) + np.uint8(3)).tobytes()
    del pat
    v3 = bytes(range(256)) * (200 << 12)   # 200 MiB
    recs = [(b"a0", b"x"), (b"a1", b"yy"), (b"a2", b""), (b"b", v1), (b"c", v2), (b"d", b"small"), (b"e", v3),
            (b"f", b"tail")]
    # Writer::insert flushes before a record when the estimate + the record reaches the block
    # size (src/writer.rs:125-130): 4.4e9 keeps b, c, d in one block (> u32::MAX bytes: u64
    # restarts) and starts a second, ordinary block at e
    w = Writer(4_400_000_000, 16)
    for k, v in recs:
        w.insert(k, v)
    return w.into_inner(), recs


def test_block_over_4gib(oracle):
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    if torch.cuda.get_device_properties(0).total_memory < (40 << 30):
        pytest.skip("needs ~40 GiB of device memory")
    import time
    from mtblx import reader
    t0 = time.time()

    def note(msg):   # progress on stdout (a long silent GPU run reads as hung)
        print(f"[{time.time() - t0:6.1f}s] {msg}", flush=True)

    data, recs = _file()
    note(f"file written: {len(data)} bytes")
    nblk = None
    for verify in (True, False):
        exp = oracle.file_scan(data, "iter", verify=verify)
        note(f"oracle scan (verify={verify}) done")
        r = reader.ReaderBuilder().verify_checksums(verify).read(data)
        off, ln, st = r._framing()
        nblk = int(st.numel())
        assert int(st[0].item()) == 2 and nblk == 2   # DIR_UNSUPPORTED: the big block, then a small one
        s = r.iter()
        assert (s.end, exp["end"]) == (reader.END_NONE, 0)
        got = s.records()
        assert [k for k, _ in got] == [k for k, _ in exp["records"]] == [k for k, _ in recs]
        assert got == exp["records"]
        note(f"device Reader (verify={verify}) bit-exact")
        del got, exp, s, r
        torch.cuda.empty_cache()
    # Reader::get into the big block (device index seek -> block seek on the u64 restart array)
    r = reader.ReaderBuilder().verify_checksums(False).read(data)
    assert r.get(b"a1") == b"yy" and r.get(b"d") == b"small" and r.get(b"b0") is None
    assert r.get(b"c") == recs[4][1]
    note("get ok")
    # a corrupted byte inside the big block: the checksum assert panics (verify on)
    d2 = bytearray(data)
    d2[1000] ^= 0x55
    e2 = oracle.file_scan(bytes(d2), "iter", verify=True)
    s2 = reader.ReaderBuilder().verify_checksums(True).read(bytes(d2)).iter()
    assert s2.end == e2["end"] == reader.END_PANIC and s2.nrec == len(e2["records"]) == 0


def test_compressed_blocks_over_4gib(oracle):
    """Zstd (CompressionType::Zstd, src/compression.rs:140-156): a block whose DECOMPRESSED content
    is >= 4 GiB (patterned values: stored small) and a block whose STORED content is >= 4 GiB
    (random values: zstd stores them raw), each Block::init'ed on its u64 restart array
    (src/block.rs:25-42) -- decompressed on the host (Reader::block, src/reader.rs:166-170) and
    decoded on the device by the emitting block seek -- against the oracle's restatement."""
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    if torch.cuda.get_device_properties(0).total_memory < (64 << 30):
        pytest.skip("needs ~64 GiB of device memory")
    import time
    from mtblx import _lib, reader
    from mtblx.writer import Writer
    if not _lib.lib().mtblx_codec_available(5):
        pytest.skip("no libzstd.so.1")
    t0 = time.time()

    def note(msg):
        print(f"[{time.time() - t0:6.1f}s] {msg}", flush=True)

    vlen = (1 << 31) + 4099
    pat = np.tile(np.arange(256, dtype=np.uint8), vlen // 256 + 1)[:vlen]
    rng = np.random.default_rng(7)
    recs = [(b"a0", b"x"), (b"b", pat.tobytes()), (b"c", (pat * np.uint8(3)).tobytes()), (b"d", b"small"),
            (b"e", rng.integers(0, 256, vlen, dtype=np.uint8).tobytes()),
            (b"f", rng.integers(0, 256, vlen, dtype=np.uint8).tobytes()), (b"g", b"tail")]
    del pat
    w = Writer(4_400_000_000, 16, 5, 1)
    for k, v in recs:
        w.insert(k, v)
    data = w.into_inner()
    note(f"file written: {len(data)} bytes")
    exp = oracle.file_scan(data, "iter", verify=True)
    note("oracle scan done")
    assert [k for k, _ in exp["records"]] == [k for k, _ in recs]
    r = reader.ReaderBuilder().verify_checksums(True).read(data)
    _, ln, st = r._framing()
    sts = st.cpu().numpy().tolist()
    assert sts[0] == 0 and sts[1] == 2, sts    # block 0 stored small (decompressed >= 4 GiB); block 1 stored >= 4 GiB
    s = r.iter()
    assert (s.end, exp["end"]) == (reader.END_NONE, 0)
    got = s.records()
    assert got == exp["records"]
    note("device Reader bit-exact")
    del got, s
    torch.cuda.empty_cache()
    # Reader::get and the stateful iterator into both blocks (compressed files: seek-based)
    assert r.get(b"d") == b"small" and r.get(b"a1") is None
    it = r.into_iter("from", b"c")
    k1, _ = it.next()
    assert k1 == b"c"
    it.seek(b"e")
    nxt = it.next()
    exp2 = oracle.iter_script(data, "from", b"c", b"", [1, ("seek", b"e"), 1], verify=True)
    assert nxt == exp2["records"][1]
    note("get / seek ok")


def test_copy_ranges_and_deferred_values(oracle):
    """r05: the values of blocks >= 4 GiB are moved by the whole grid (mtblx_block_seek_batch_ex
    leaves them to mtblx_copy_ranges) instead of the seeking wave.  mtblx_copy_ranges on ragged,
    unaligned ranges (0..40 B and MiBs) equals the host copy; the deferred emission (small_caps,
    and values=False for key capacities) equals the wave-copied one on ordinary blocks."""
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import ctypes as C
    import corpus
    from mtblx import _lib, codec, iterator
    rng = np.random.default_rng(5)
    src = rng.integers(0, 256, 12 << 20, dtype=np.uint8)
    lens = [int(x) for x in rng.integers(0, 41, 200)] + [3 << 20, (1 << 20) + 7, 17, 0, 4099]
    so = [int(rng.integers(0, src.size - n + 1)) for n in lens]
    do, acc = [], 5
    for n in lens:
        do.append(acc)
        acc += n + int(rng.integers(0, 3))
    dst = np.zeros(acc + 16, np.uint8)
    ch = [(n + 15) // 16 for n in lens]
    cb = np.concatenate([[0], np.cumsum(ch)[:-1]]).astype(np.int64)
    t = lambda a: torch.tensor(np.asarray(a, np.int64), device="cuda")   # noqa: E731
    ds, dd = torch.from_numpy(src).to("cuda"), torch.from_numpy(dst).to("cuda")
    args = [t(so), t(do), t(lens), t(cb)]
    rc = _lib.lib().mtblx_copy_ranges(C.c_void_p(ds.data_ptr()), C.c_void_p(args[0].data_ptr()),
                                      C.c_void_p(dd.data_ptr()), C.c_void_p(args[1].data_ptr()),
                                      C.c_void_p(args[2].data_ptr()), C.c_void_p(args[3].data_ptr()), len(lens),
                                      int(sum(ch)), C.c_void_p(codec._stream_handle(None)))
    assert rc == 0
    for a, b, n in zip(so, do, lens):
        dst[b: b + n] = src[a: a + n]
    assert np.array_equal(dd.cpu().numpy(), dst)
    # deferred emission == the wave's own copies
    for seed in (1, 2):
        recs = corpus.random_records(np.random.default_rng(seed), 300, 0, 40, 0, 5000)
        blk = oracle.build_block(recs, restart_interval=16)
        d = torch.frombuffer(bytearray(b"\x00" * 3 + blk), dtype=torch.uint8).to("cuda")
        content = (d, 3, len(blk))
        a = iterator.block_seek(content, None)
        b = iterator.block_seek(content, None, small_caps=True)
        c = iterator.block_seek(content, None, values=False)
        assert a.host_records() == b.host_records() == recs
        assert torch.equal(a.kcaps, c.kcaps) and torch.equal(a.key_end, c.key_end) and torch.equal(a.val_end, c.val_end)
