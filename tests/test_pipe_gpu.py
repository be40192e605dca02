"""End-to-end host -> device -> host decode (mtblx_pipe_decode) and snappy files on the GPU,
bit-exact against the oracle.

Parity anchors: uncompressed blocks -> oracle_decode_blocks on the same bytes; snappy files
-> the oracle's decode of the None-compressed file the same records produce (the flush rule
runs on uncompressed sizes, so both files cut identical blocks) and the oracle's ReaderIntoIter
restatement, which decompresses with its own snappy decoder.
"""
import numpy as np
import pytest

import corpus

pytestmark = pytest.mark.gpu


def _need_gpu():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


def _files(recs, block_size=4096, interval=16):
    from mtblx.writer import Writer
    out = {}
    for comp in (0, 1):
        w = Writer(block_size, interval, comp)
        w.insert_batch(*recs) if isinstance(recs, tuple) else [w.insert(k, v) for k, v in recs]
        data = w.into_inner_np() if isinstance(recs, tuple) else np.frombuffer(w.into_inner(), np.uint8).copy()
        off, ln = w.block_dir
        out[comp] = (data, off, ln)
    return out


def _cfg2_records(nblk):
    from mtblx import synth
    per = (4096 - 64) // 79
    nrec = nblk * per
    keys, vals, kl, vl = synth.cfg2_arrays(nrec)
    ke = np.arange(1, nrec + 1, dtype=np.uint64) * np.uint64(kl)
    ve = np.arange(1, nrec + 1, dtype=np.uint64) * np.uint64(vl)
    return keys, ke, vals, ve


def _pipe_decode(data, off, ln, comp, exp, chunk=1 << 20, max_blocks=1 << 16, pinned_src=False, caps=None,
                 device_snappy=False):
    from mtblx import pipe
    p = pipe.HostPipe(chunk_bytes=chunk, max_blocks=max_blocks, threads=8, device_snappy=device_snappy)
    nr = int(exp.nrec.sum())
    caps = caps or (nr, exp.keys.size, exp.vals.size)
    out = pipe.HostOutputs(off.size, *caps)
    if pinned_src:
        pipe.register(data)
    try:
        stats = p.decode(data, off, ln, out, compression=comp)
    finally:
        if pinned_src:
            pipe.unregister(data)
    return out, stats


def _assert_same(out, exp):
    n = exp.nrec.size
    assert np.array_equal(out.status[:n], exp.status)
    assert np.array_equal(out.nrec[:n], exp.nrec)
    assert np.array_equal(out.rec_base[:n], exp.rec_base)
    assert np.array_equal(out.key_base[:n], exp.key_base)
    assert np.array_equal(out.val_base[:n], exp.val_base)
    nr = int(exp.nrec.sum())
    assert tuple(int(x) for x in out.totals[:3]) == (nr, exp.keys.size, exp.vals.size)
    assert np.array_equal(out.key_end[:nr], exp.key_end)
    assert np.array_equal(out.val_end[:nr], exp.val_end)
    assert np.array_equal(out.keys[: exp.keys.size], exp.keys)
    assert np.array_equal(out.vals[: exp.vals.size], exp.vals)


def test_pipe_uncompressed_chunks(oracle):
    """many chunks (small chunk size and block cap), pageable and pinned sources"""
    _need_gpu()
    from mtblx import synth
    data, off, ln = synth.cfg2_file(2000)
    exp = oracle.decode_blocks(data, off, ln)
    for chunk, mb, pinned in ((1 << 20, 1 << 16, False), (256 << 10, 37, False), (300_000, 1000, True),
                              (64 << 20, 1 << 16, True)):
        out, st = _pipe_decode(data, off, ln, 0, exp, chunk=chunk, max_blocks=mb, pinned_src=pinned)
        _assert_same(out, exp)
        assert int(out.totals[3]) == 0
        assert st.block_bytes == int(ln.sum()) and st.decompress_errors == 0


def test_pipe_mixed_and_odd_blocks(oracle):
    """builder blocks of every shape + mutated blocks (all statuses), 64 KiB blocks, gaps"""
    _need_gpu()
    rng = np.random.default_rng(3)
    blocks = corpus.builder_blocks(oracle, seed=31, count=150, max_bytes=8000)
    blocks += corpus.mutated_blocks(oracle, seed=32, count=200)
    for _ in range(4):
        recs = corpus.random_records(rng, 600, 8, 200, 64, 64)
        b = oracle.build_block(recs)
        if len(b) < 65000:
            blocks.append(b)
    data, off, ln = corpus.pack(blocks, rng=rng, lead=5)
    exp = oracle.decode_blocks(data, off, ln)
    out, _ = _pipe_decode(data, off, ln, 0, exp, chunk=200_000, max_blocks=64)
    _assert_same(out, exp)


def test_pipe_key_expansion_regrows_slot(oracle):
    """keys far longer than the block bytes (long shared prefixes, empty values): the chunk's
    device outputs overflow the slot's 2x estimate and the chunk is decoded again exactly"""
    _need_gpu()
    base = b"k" * 240
    recs = [(base + i.to_bytes(4, "big"), b"") for i in range(20000)]
    f = _files(recs, block_size=4096)
    data, off, ln = f[0]
    exp = oracle.decode_blocks(data, off, ln)
    assert exp.keys.size > 4 * int(ln.sum())
    out, _ = _pipe_decode(data, off, ln, 0, exp, chunk=1 << 20)
    _assert_same(out, exp)


def test_pipe_snappy_equals_uncompressed(oracle):
    _need_gpu()
    f = _files(_cfg2_records(400))
    d0, o0, l0 = f[0]
    d1, o1, l1 = f[1]
    assert o0.size == o1.size   # cfg2 keys/values are random bytes: snappy barely changes the size
    exp = oracle.decode_blocks(d0, o0, l0)
    for chunk in (1 << 20, 100_000):
        out, st = _pipe_decode(d1, o1, l1, 1, exp, chunk=chunk)
        _assert_same(out, exp)
        assert st.block_bytes == int(l0.sum()) and st.decompress_errors == 0


def test_pipe_device_snappy_equals_uncompressed(oracle):
    """MTBLX_PIPE_DEVICE_SNAPPY: stored (compressed) bytes cross PCIe and are decompressed on
    the device; same outputs as the None file, pageable and pinned sources, several chunkings;
    plus a compressible file (repeated values, ratio well above 1)"""
    _need_gpu()
    from mtblx import pipe
    f = _files(_cfg2_records(400))
    d0, o0, l0 = f[0]
    d1, o1, l1 = f[1]
    exp = oracle.decode_blocks(d0, o0, l0)
    for chunk, pinned in ((1 << 20, False), (100_000, True), (64 << 20, True)):
        out, st = _pipe_decode(d1, o1, l1, 1, exp, chunk=chunk, pinned_src=pinned, device_snappy=True)
        _assert_same(out, exp)
        assert st.block_bytes == int(l0.sum()) and st.decompress_errors == 0
        assert st.h2d_bytes < int(l1.sum()) + 40 * o1.size + 4096
    from mtblx import synth
    f = _files(list(synth.cfg1_records(20000)), block_size=8192)
    d0, o0, l0 = f[0]
    d1, o1, l1 = f[1]
    assert int(l1.sum()) * 3 < int(l0.sum())
    exp = oracle.decode_blocks(d0, o0, l0)
    for chunk in (1 << 20, 200_000):
        out, st = _pipe_decode(d1, o1, l1, 1, exp, chunk=chunk, device_snappy=True)
        _assert_same(out, exp)
        assert st.decompress_errors == 0 and st.h2d_bytes < int(l0.sum()) // 2


def test_pipe_snappy_corrupt_block(oracle):
    """a block that fails decompression -> MTBLX_ST_DECOMPRESS (the reference: Err(Error::Io)),
    every other block decoded; host and device decompression alike"""
    _need_gpu()
    f = _files(_cfg2_records(60))
    d0, o0, l0 = f[0]
    d1, o1, l1 = f[1]
    d1 = d1.copy()
    bad = [3, 40]
    for b in bad:
        d1[int(o1[b]) + int(l1[b]) - 1] ^= 0xFF   # last literal byte flips: length still fine...
        d1[int(o1[b])] ^= 0x01                    # ...but the preamble length no longer matches
    d1[int(o1[50]) + int(l1[50]) // 2] ^= 0x5A   # mid-stream damage: preamble intact
    exp = oracle.decode_blocks(d0, o0, l0)
    from mtblx import pipe
    zbad = [b for b in range(o1.size) if pipe.snappy_decompress(d1[int(o1[b]): int(o1[b]) + int(l1[b])]) is None]
    assert set(bad) <= set(zbad)
    for dev in (False, True):
        out, st = _pipe_decode(d1, o1, l1, 1, exp, device_snappy=dev)
        assert st.decompress_errors == len(zbad)
        for b in range(o0.size):
            if b in zbad:
                assert out.status[b] == 6 and out.nrec[b] == 0
            elif b == 50:   # decompressed to other bytes of the right length: decoded as they are
                assert out.status[b] != 6
            else:
                assert out.status[b] == 0 and out.nrec[b] == exp.nrec[b]


def test_pipe_capacity_overflow_reports_sizes(oracle):
    _need_gpu()
    from mtblx import synth
    data, off, ln = synth.cfg2_file(300)
    exp = oracle.decode_blocks(data, off, ln)
    nr = int(exp.nrec.sum())
    out, _ = _pipe_decode(data, off, ln, 0, exp, chunk=64 << 10, caps=(nr, exp.keys.size // 2, exp.vals.size))
    assert int(out.totals[3]) & 1
    assert tuple(int(x) for x in out.totals[:3]) == (nr, exp.keys.size, exp.vals.size)
    st = out.status[: off.size]
    assert (st == 5).any() and st[0] == 0
    first_bad = int(np.nonzero(st == 5)[0][0])
    assert (st[first_bad:] == 5).all()
    kb = int(exp.key_base[first_bad])
    assert np.array_equal(out.keys[:kb], exp.keys[:kb])


def test_reader_snappy_files(oracle):
    """device Reader over snappy files (host decompression, device decode) == the oracle's
    ReaderIntoIter restatement (its own snappy decoder), including a corrupted block"""
    _need_gpu()
    from mtblx import reader
    rng = np.random.default_rng(51)
    recs = corpus.random_records(rng, 2500, 0, 50, 0, 150)
    f = _files(recs, block_size=2048, interval=8)
    d1 = f[1][0].tobytes()
    for data, verify in ((d1, True), (d1, False)):
        exp = oracle.file_scan(data, "iter", verify=verify)
        s = reader.ReaderBuilder().verify_checksums(verify).read(data).iter()
        assert s.end == exp["end"] and s.records() == exp["records"] == recs
    # corrupt one block's snappy stream (CRC not verified) -> Err(Io) after its predecessors
    o1, l1 = f[1][1], f[1][2]
    d = bytearray(d1)
    d[int(o1[5])] ^= 0x01
    exp = oracle.file_scan(bytes(d), "iter", verify=False)
    s = reader.ReaderBuilder().verify_checksums(False).read(bytes(d)).iter()
    assert exp["end"] == reader.END_ERR_NEXT and exp["err"] == "Io"
    assert s.end == exp["end"] and s.err == "Io" and s.records() == exp["records"]
    r = reader.ReaderBuilder().read(d1)
    k, v = recs[1234]
    assert r.get(k) == v and r.get(k + b"\x00") is None
