"""f3 device Reader (index -> directory -> checksum -> decode on the GPU) vs the oracle's
restatement of ReaderBuilder::read + ReaderIntoIter (oracle_file_scan)."""
import numpy as np
import pytest

import corpus

pytestmark = pytest.mark.gpu


def _reader():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from mtblx import reader
    return reader


def _write(records, block_size=4096, interval=16):
    from mtblx.writer import Writer
    w = Writer(block_size, interval)
    for k, v in records:
        w.insert(k, v)
    return w.into_inner()


def _check(oracle, data: bytes, verify=True):
    rd = _reader()
    exp = oracle.file_scan(data, "iter", verify=verify)
    try:
        r = rd.ReaderBuilder().verify_checksums(verify).read(data)
    except rd.MtblError as e:
        assert exp["end"] == rd.END_ERR_OPEN and exp["err"] == str(e), (exp["end"], exp["err"], e)
        return exp
    except rd.ReferencePanic:
        assert exp["end"] == rd.END_PANIC
        return exp
    s = r.iter()
    assert s.end == exp["end"], (s.end, exp["end"], exp["err"])
    got = s.records()
    assert len(got) == len(exp["records"]), (len(got), len(exp["records"]))
    assert got == exp["records"]
    return exp


def test_cfg1_file(oracle):
    from mtblx import synth
    data = _write(list(synth.cfg1_records()))
    exp = _check(oracle, data)
    assert len(exp["records"]) == 10_000


def test_random_files(oracle):
    rng = np.random.default_rng(31)
    for bs, iv, n in ((1024, 1, 300), (4096, 16, 2000), (16384, 4, 3000), (65536, 16, 4000), (8192, 40, 1500)):
        recs = corpus.random_records(rng, n, 0, 80, 0, 200)
        _check(oracle, _write(recs, bs, iv))
    _check(oracle, _write([]))                      # empty file: index with no entries


def test_corrupted_files(oracle):
    """stored checksum flips, content flips with and without verification, index entries
    pointing past the end of the file"""
    rd = _reader()
    from mtblx import synth
    rng = np.random.default_rng(32)
    data, off, ln = synth.cfg2_file(40)
    raw = bytes(data)
    seen = set()
    for trial in range(40):
        d = bytearray(raw)
        kind = trial % 4
        b = int(rng.integers(0, off.size))
        if kind == 0:                                   # stored crc of block b
            d[int(off[b]) - 3] ^= 0x10
        elif kind == 1:                                 # a content byte of block b
            d[int(off[b]) + int(rng.integers(0, int(ln[b])))] ^= 1 << int(rng.integers(0, 8))
        elif kind == 2:                                 # restart count of block b
            e = int(off[b]) + int(ln[b])
            d[e - 4:e] = int(rng.integers(0, 1 << 32)).to_bytes(4, "little")
        else:                                           # header byte of block b's first entry
            d[int(off[b]) + 1] ^= 0x80
        for verify in (True, False):
            exp = _check(oracle, bytes(d), verify=verify)
            seen.add(exp["end"])
    assert rd.END_PANIC in seen and rd.END_NONE in seen


def _check_get(oracle, data: bytes, queries, verify=True):
    rd = _reader()
    from mtblx import _lib
    r = rd.ReaderBuilder().verify_checksums(verify).read(data)
    st, vo, vl = r.get_batch(queries)
    st = st.cpu().numpy()
    vo = vo.cpu().numpy()
    vl = vl.cpu().numpy()
    src = data if r.compression == 0 else r.value_source.cpu().numpy().tobytes()   # decompressed blocks
    end_of = {rd.END_NONE: _lib.GET_NONE, rd.END_PANIC: _lib.GET_PANIC, rd.END_ERR_OPEN: _lib.GET_ERR,
              rd.END_ERR_NEXT: _lib.GET_ERR, rd.END_LOOP: _lib.GET_LOOP}
    for q, key in enumerate(queries):
        exp = oracle.file_scan(data, "get", key=key, verify=verify)
        if exp["records"]:
            assert exp["end"] == rd.END_NONE
            assert st[q] == _lib.GET_FOUND, (q, key, st[q])
            assert src[vo[q]: vo[q] + vl[q]] == exp["records"][0][1]
        else:
            assert st[q] == end_of[exp["end"]], (q, key, st[q], exp["end"])


def test_get_batch_valid_files(oracle):
    rng = np.random.default_rng(41)
    for bs, iv, n in ((1024, 1, 200), (4096, 16, 1500), (65536, 16, 3000), (8192, 3, 800)):
        recs = corpus.random_records(rng, n, 0, 40, 0, 100)
        data = _write(recs, bs, iv)
        keys = [k for k, _ in recs]
        qs = [keys[int(i)] for i in rng.integers(0, n, 150)]                      # hits
        qs += [k + b"\x00" for k in qs[:40]] + [k[:-1] for k in qs[:40] if k]   # near misses
        qs += [b"", b"\xff" * 50, keys[0], keys[-1], keys[-1] + b"\x01"]
        _check_get(oracle, data, qs)


def test_get_batch_corrupted(oracle):
    from mtblx import synth
    rng = np.random.default_rng(42)
    data, off, ln = synth.cfg2_file(30)
    raw = bytes(data)
    recs = oracle.file_scan(raw, "iter")["records"]
    for trial in range(16):
        d = bytearray(raw)
        b = int(rng.integers(0, off.size))
        if trial % 3 == 0:
            d[int(off[b]) - 3] ^= 0x10                                       # stored crc
        elif trial % 3 == 1:
            d[int(off[b]) + int(rng.integers(0, int(ln[b])))] ^= 0xA5          # content byte
        else:
            e = int(off[b]) + int(ln[b])
            d[e - 8:e - 4] = int(rng.integers(0, 1 << 32)).to_bytes(4, "little")   # a restart point
        qs = [recs[int(i)][0] for i in rng.integers(0, len(recs), 40)] + [b"", b"\xff" * 20]
        for verify in (True, False):
            _check_get(oracle, bytes(d), qs, verify=verify)


@pytest.mark.parametrize("comp", [1, 2, 5])
def test_get_batch_compressed(oracle, comp):
    """the batched Reader::get on Snappy / Zlib / Zstd files (mtblx_get_decompressed: framing and
    checksum on the stored bytes, the scan on the host-decompressed blocks), valid files and
    files with a corrupted stored block (Err(Io) / checksum panic), verify on and off"""
    rng = np.random.default_rng(43 + comp)
    from mtblx.writer import Writer
    for bs, iv, n in ((1024, 4, 400), (4096, 16, 2500)):
        recs = corpus.random_records(rng, n, 0, 40, 0, 200)
        w = Writer(bs, iv, comp)
        for k, v in recs:
            w.insert(k, v)
        data = w.into_inner()
        off, ln = w.block_dir
        keys = [k for k, _ in recs]
        qs = [keys[int(i)] for i in rng.integers(0, n, 120)]
        qs += [k + b"\x00" for k in qs[:30]] + [b"", b"\xff" * 30, keys[0], keys[-1], keys[-1] + b"\x01"]
        _check_get(oracle, data, qs)
        for b in (1, len(off) // 2):
            d = bytearray(data)
            d[int(off[b]) + int(ln[b]) // 2] ^= 0x5A            # a stored byte: checksum / codec error
            for verify in (True, False):
                _check_get(oracle, bytes(d), qs[:60] + [keys[-1]], verify=verify)


def _index_entry_offsets(data: bytes):
    """(content start, entry offsets, restart points) of a V2 file's index block, every header a
    1-byte varint triple (host walk for building corrupt files)"""
    meta0 = int.from_bytes(data[-512:-504], "little")
    p, ln, sh = meta0, 0, 0
    while True:
        b = data[p]
        ln |= (b & 0x7F) << sh
        p += 1
        sh += 7
        if b < 0x80:
            break
    c0 = p + 4
    content = data[c0: c0 + ln]
    n = int.from_bytes(content[-4:], "little")
    R = ln - 4 * (n + 1)
    restarts = [int.from_bytes(content[R + 4 * i: R + 4 * i + 4], "little") for i in range(n)]
    offs, q = [], restarts[0]
    while q < R:
        offs.append(q)
        assert content[q] < 128 and content[q + 1] < 128 and content[q + 2] < 128
        q += 3 + content[q + 1] + content[q + 2]
    return c0, offs, restarts


@pytest.mark.parametrize("comp", [1, 2, 5])
def test_get_batch_compressed_seek_past_linear_walk(oracle, comp):
    """on a compressed file whose index is corrupt mid-chain (read with
    verification off), the linear walk of the index (the directory, mtblx_block_dir) stops at
    the corrupt entry, while Reader::get's index seek jumps over it through later restart
    points and lands on blocks the walk never reached.  The reference reads, decompresses and
    scans those blocks (src/reader.rs:111-122, :140-172); mtblx_get_decompressed reports them
    MTBLX_GET_MISSING and get_batch decompresses them and runs the batch again -- the results
    equal the oracle's, where the earlier library answered Err(Io)."""
    rng = np.random.default_rng(90 + comp)
    from mtblx.writer import Writer
    recs = corpus.random_records(rng, 3000, 8, 40, 40, 120)
    w = Writer(1024, 16, comp)
    for k, v in recs:
        w.insert(k, v)
    data = w.into_inner()
    c0, offs, restarts = _index_entry_offsets(data)
    assert len(restarts) >= 4
    bad_entry = offs.index(restarts[1]) + 3               # inside the second restart interval
    d = bytearray(data)
    d[c0 + offs[bad_entry]] = 0x7F                        # shared 127 > the key Vec's capacity: panic
    keys = [k for k, _ in recs]
    qs = [keys[int(i)] for i in rng.integers(0, len(keys), 150)] + [keys[-1], keys[0], keys[-1] + b"\x01"]
    rd = _reader()
    r = rd.ReaderBuilder().verify_checksums(False).read(bytes(d))
    ntab0 = r._dec_table()[4]
    assert ntab0 <= bad_entry                              # the linear walk stopped at the corruption
    _check_get(oracle, bytes(d), qs, verify=False)
    r.get_batch(qs)
    assert r._dec_table()[4] > ntab0                       # blocks past the corruption were added


def test_get_stale_value_when_next_block_invalid(oracle):
    """Reader::get whose seek runs past a block while the NEXT block fails Block::init
    returns Ok(Some(value of the last entry the seek parsed in the old block)) -- the crate's
    match on Some(_) (src/reader.rs:111-122) -- not an error."""
    from mtblx import synth
    data, off, ln = synth.cfg2_file(30)
    raw = bytearray(bytes(data))
    b = 11
    e = int(off[b]) + int(ln[b])
    for n in (0xFFFFFFFF, 0x80000000, 0x40000001, 0x3FFFFFFF, int(ln[b]) // 4 + 1):
        blk = bytes(raw[int(off[b]):e - 4]) + n.to_bytes(4, "little")
        if oracle.decode_block(blk)[0] == 1:       # Block::init -> None (InvalidBlock)
            raw[e - 4:e] = n.to_bytes(4, "little")
            break
    else:
        pytest.skip("no restart count gives InvalidBlock for this block")
    recs = oracle.file_scan(bytes(data), "iter")["records"]
    prev_last = [k for k, _ in recs][:int(synth.cfg2_file.last_block_nrec[:b].sum())][-1]
    qs = [prev_last + b"\x00", prev_last + b"\x00\x01", prev_last, recs[0][0]]
    stale = oracle.file_scan(bytes(raw), "get", key=qs[0], verify=False)
    assert stale["end"] == 0 and len(stale["records"]) == 1    # Ok(Some(stale value))
    _check_get(oracle, bytes(raw), qs, verify=False)
