"""Seek-based iteration on the GPU: Reader::iter_from / iter_prefix /
iter_range (src/reader.rs:128-138) and the stateful ReaderIntoIter with next() / seek()
(:219-405), against the oracle's restatement (oracle_file_scan modes from / prefix / range and
oracle_iter_script, which pins the block_offset quirk of ReaderIntoIter::seek).

Files: product Writer output (raw and zlib), plus corrupted copies -- restart entries with
shared != 0 (BlockIter::seek's early return, src/block.rs:167-170) and random byte flips --
read with verification off so the corruption reaches the block scan."""
import numpy as np
import pytest

import corpus

pytestmark = pytest.mark.gpu


def _mods():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from mtblx import reader
    return reader


def _write(records, bs=1024, iv=4, comp=0):
    from mtblx.writer import Writer
    w = Writer(bs, iv, comp, 1)
    for k, v in records:
        w.insert(k, v)
    return w.into_inner(), w.block_dir


def _probe_keys(rng, recs, n=24):
    keys = [k for k, _ in recs]
    out = [b"", b"\x00", b"\xff" * 8]
    for _ in range(n):
        k = keys[int(rng.integers(0, len(keys)))]
        c = int(rng.integers(0, 4))
        if c == 0:
            out.append(k)                                   # present
        elif c == 1:
            out.append(k + b"\x00")                         # just after
        elif c == 2:
            out.append(k[: max(0, len(k) - 1)])             # a prefix
        else:
            out.append(k[:-1] + bytes([(k[-1] + 1) & 0xFF]) if k else b"\x01")
    return out


def _bulk_check(oracle, data, verify, rng, recs):
    rd = _mods()
    try:
        r = rd.ReaderBuilder().verify_checksums(verify).read(data)
    except (rd.MtblError, rd.ReferencePanic):
        return 0
    keys = _probe_keys(rng, recs)
    n = 0
    for k in keys:
        for mode, k1, k2 in (("from", k, b""), ("prefix", k[:3], b""), ("prefix", k, b""),
                             ("range", k, k + b"\xff"), ("range", k[:2], k)):
            exp = oracle.file_scan(data, mode, k1, k2, verify=verify)
            s = {"from": lambda: r.iter_from(k1), "prefix": lambda: r.iter_prefix(k1),
                 "range": lambda: r.iter_range(k1, k2)}[mode]()
            assert (s.end, s.err if s.end in (rd.END_ERR_OPEN, rd.END_ERR_NEXT) else None) == \
                (exp["end"], exp["err"] if exp["end"] in (rd.END_ERR_OPEN, rd.END_ERR_NEXT) else None), (mode, k1, k2)
            assert s.records() == exp["records"], (mode, k1, k2, s.nrec, len(exp["records"]))
            n += 1
    return n


@pytest.mark.parametrize("bs,iv,comp", [(1024, 4, 0), (4096, 16, 0), (256, 1, 0), (2048, 3, 2)])
def test_bulk_valid_files(oracle, bs, iv, comp):
    rng = np.random.default_rng(bs + iv + comp)
    recs = corpus.random_records(rng, 4000, 0, 30, 0, 120)
    data, _ = _write(recs, bs, iv, comp)
    for verify in (True, False):
        assert _bulk_check(oracle, data, verify, rng, recs) > 100


def test_bulk_touches_only_needed_blocks(oracle):
    """iter_prefix on a narrow range decodes a handful of blocks, not the file"""
    rd = _mods()
    from mtblx import iterator
    recs = [(b"k%06d" % i, b"v" * (i % 50)) for i in range(60000)]
    data, (off, _) = _write(recs, 1024, 16)
    r = rd.Reader(data)
    seen = []
    orig = r._walk_range

    def spy(i0, i1):
        seen.append((i0, i1))
        return orig(i0, i1)

    r._walk_range = spy
    s = r.iter_prefix(b"k03001")
    assert s.records() == [x for x in recs if x[0].startswith(b"k03001")]
    assert sum(b - a for a, b in seen) <= 4 and off.size > 1000
    assert r._dir is None        # no whole-file checksum pass either
    assert iterator.prefix_successor(b"a\xff\xff") == b"b" and iterator.prefix_successor(b"\xff") is None


def _corrupt_restart_shared(data, off, ln, rng, nblk=6):
    """set shared = 1 in the entry at a middle restart point of some data blocks"""
    d = bytearray(data)
    for b in rng.choice(off.size, size=min(nblk, off.size), replace=False):
        o, L = int(off[b]), int(ln[b])
        blk = d[o: o + L]
        nr = int.from_bytes(blk[L - 4:], "little")
        if nr < 3:
            continue
        ro = L - 4 * (nr + 1)
        mid = int(rng.integers(1, nr))
        p = int.from_bytes(blk[ro + 4 * mid: ro + 4 * mid + 4], "little")
        if p + 3 < ro and blk[p] == 0 and blk[p + 1] < 128 and blk[p + 2] < 128:
            d[o + p] = 1
    return bytes(d)


@pytest.mark.parametrize("seed", [1, 2])
def test_bulk_corrupt_restart_shared(oracle, seed):
    rng = np.random.default_rng(40 + seed)
    recs = corpus.random_records(rng, 3000, 1, 24, 0, 60)
    data, (off, ln) = _write(recs, 1024, 4)
    bad = _corrupt_restart_shared(data, off, ln, rng, 12)
    assert bad != data
    assert _bulk_check(oracle, bad, False, rng, recs) > 50


def test_bulk_random_corruption(oracle):
    rng = np.random.default_rng(77)
    recs = corpus.random_records(rng, 1500, 0, 20, 0, 40)
    data, (off, ln) = _write(recs, 512, 2)
    for t in range(6):
        d = bytearray(data)
        for _ in range(4):
            b = int(rng.integers(0, off.size))
            d[int(off[b]) + int(rng.integers(0, int(ln[b])))] ^= int(rng.integers(1, 256))
        _bulk_check(oracle, bytes(d), False, rng, recs)


def _run_script(data, verify, mode, key, key2, ops):
    rd = _mods()
    out = dict(records=[], ops=[], end=rd.END_NONE, err=None)
    try:
        r = rd.ReaderBuilder().verify_checksums(verify).read(data)
        it = r.into_iter(mode, key, key2)
    except rd.MtblError as e:
        out.update(end=rd.END_ERR_OPEN, err=str(e))
        return out
    except rd.ReferencePanic:
        out["end"] = rd.END_PANIC
        return out
    except rd.ReferenceLoop:
        out["end"] = rd.END_LOOP
        return out
    try:
        for op in ops:
            if isinstance(op, int):
                n, code = 0, 0
                for _ in range(op):
                    try:
                        rec = it.next()
                    except rd.MtblError as e:
                        code = 2
                        out["err"] = str(e)
                        break
                    if rec is None:
                        code = 1
                        break
                    out["records"].append(rec)
                    n += 1
                out["ops"].append((n, code))
            else:
                try:
                    it.seek(op[1])
                    out["ops"].append((0, 0))
                except rd.MtblError as e:
                    out["ops"].append((0, 2))
                    out["err"] = str(e)
    except rd.ReferencePanic:
        out["end"] = rd.END_PANIC
    except rd.ReferenceLoop:
        out["end"] = rd.END_LOOP
    return out


def _script_check(oracle, data, verify, mode, key, key2, ops):
    got = _run_script(data, verify, mode, key, key2, ops)
    exp = oracle.iter_script(data, mode, key, key2, ops, verify=verify)
    assert got["end"] == exp["end"], (mode, key, ops, got["end"], exp["end"])
    assert got["records"] == exp["records"], (mode, key, ops)
    nops = len(got["ops"])
    assert got["ops"] == exp["ops"][:nops], (got["ops"], exp["ops"])
    if exp["end"] == 0 and any(c == 2 for _, c in exp["ops"]):
        assert got["err"] == exp["err"]
    return exp


def test_stateful_seek_quirk(oracle):
    """seek back into the first block after new_from: block_offset is still 0 and block 0's
    offset is 0, so the reference re-seeks the block it holds (not block 0)"""
    recs = [(b"k%05d" % i, b"v%d" % i) for i in range(3000)]
    data, _ = _write(recs, 512, 4)
    ops = [3, ("seek", b"k00002"), 2, ("seek", b"k02999"), 5, ("seek", b"zzz"), 3, ("seek", b"k00500"), 4]
    exp = _script_check(oracle, data, True, "from", b"k01000", b"", ops)
    assert exp["records"][3][0] != b"k00002"          # the quirk is really exercised
    _script_check(oracle, data, True, "iter", b"", b"", [10, ("seek", b"k00003"), 3, 400, ("seek", b"k01500"), 2])
    _script_check(oracle, data, False, "prefix", b"k001", b"", [50, ("seek", b"k0019"), 30, 200])
    _script_check(oracle, data, True, "range", b"k00100", b"k00400", [20, ("seek", b"k00390"), 50])
    _script_check(oracle, data, True, "get", b"k00300", b"", [5, ("seek", b"k00300"), 5])


@pytest.mark.parametrize("comp", [0, 2])
def test_stateful_random_scripts(oracle, comp):
    rng = np.random.default_rng(90 + comp)
    recs = corpus.random_records(rng, 2500, 0, 24, 0, 90)
    data, (off, ln) = _write(recs, 700, 3, comp)
    files = [(data, True)]
    if comp == 0:
        files.append((_corrupt_restart_shared(data, off, ln, rng, 10), False))
    for d, verify in files:
        for t in range(12):
            keys = _probe_keys(rng, recs, 8)
            ops = []
            for _ in range(int(rng.integers(2, 9))):
                if rng.random() < 0.45:
                    ops.append(("seek", keys[int(rng.integers(0, len(keys)))]))
                else:
                    ops.append(int(rng.choice([1, 2, 7, 40, 300])))
            mode = str(rng.choice(["iter", "from", "prefix", "range"]))
            k = keys[int(rng.integers(0, len(keys)))]
            _script_check(oracle, d, verify, mode, k if mode != "prefix" else k[:2], k + b"\x80", ops)


def _index_window(data):
    """(content offset, length) of the index block (footer -> varint64 length | crc | content)"""
    off = int.from_bytes(data[len(data) - 512: len(data) - 504], "little")
    n, sh, p = 0, 0, off
    while True:
        b = data[p]
        n |= (b & 0x7F) << sh
        sh += 7
        p += 1
        if b < 128:
            break
    return p + 4, n


def test_seek_kat_gpu(oracle):
    """the hand-derived ReaderIntoIter::seek vectors (tests/golden/kat.json seek_kat): the data
    block is seeked to the landed separator (src/reader.rs:305,328) -- equal to the last key,
    bumped, and write_u16-appended"""
    import json
    import os
    kat = json.load(open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "kat.json")))["seek_kat"]
    recs = [(k.encode(), bytes([0x41 + i]) * kat["value_len"]) for i, k in enumerate(kat["keys"])]
    data, _ = _write(recs, kat["block_size"], kat["restart_interval"])
    assert data == oracle.write_file(recs, kat["block_size"], kat["restart_interval"])
    for sc in kat["scripts"]:
        ops = [o if isinstance(o, int) else ("seek", o[1].encode()) for o in sc["ops"]]
        got = _run_script(data, True, sc["mode"], sc["key"].encode(), b"", ops)
        assert [k.decode() for k, _ in got["records"]] == sc["yields"], sc["why"]
        _script_check(oracle, data, True, sc["mode"], sc["key"].encode(), b"", ops)


def _corrupt_index(data, rng, kind):
    """a copy whose INDEX block is damaged: "restart" sets shared != 0 in entries at restart
    points (BlockIter::seek's early return on the live index iterator, src/block.rs:167-170;
    key-capacity asserts), "shared" raises shared past the previous key's length in plain
    entries (truncate no-ops: keys rebuilt from another restart differ), "bytes" flips bytes"""
    d = bytearray(data)
    o, L = _index_window(data)
    nr = int.from_bytes(d[o + L - 4: o + L], "little")
    ro = L - 4 * (nr + 1)
    if kind == "bytes":
        for _ in range(3):
            d[o + int(rng.integers(0, max(ro, 1)))] ^= int(rng.integers(1, 256))
        return bytes(d)
    rps = [int.from_bytes(d[o + ro + 4 * i: o + ro + 4 * i + 4], "little") for i in range(nr)]
    if kind == "restart":
        for i in rng.choice(nr, size=min(nr, 4), replace=False):
            p = rps[int(i)]
            if p + 3 < ro and d[o + p] == 0 and d[o + p + 1] < 128 and d[o + p + 2] < 128:
                d[o + p] = int(rng.integers(1, 12))
        return bytes(d)
    p, n = rps[0], 0                                  # walk the chain, bump some shared fields
    while p + 3 <= ro and n < 100000:
        sh, ns, vl = d[o + p], d[o + p + 1], d[o + p + 2]
        if sh >= 128 or ns >= 128 or vl >= 128:
            break
        if p not in rps and rng.random() < 0.15:
            d[o + p] = min(127, sh + int(rng.integers(1, 20)))
        p += 3 + ns + vl
        n += 1
    return bytes(d)


def _dump_failure(data, *what):
    """keep a failing corrupted file for offline analysis (gpurun_out/ travels back)"""
    import os
    d = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "gpurun_out", "failures")
    os.makedirs(d, exist_ok=True)
    n = len(os.listdir(d))
    open(os.path.join(d, f"f{n}.mtbl"), "wb").write(data)
    open(os.path.join(d, f"f{n}.txt"), "w").write(repr(what))


@pytest.mark.parametrize("kind", ["restart", "shared", "bytes"])
def test_stateful_live_index_iterator(oracle, kind):
    """ReaderIntoIter::seek re-seeks the LIVE index iterator (src/reader.rs:303): on a corrupt
    index (verification off) an early return keeps its old position and key capacity, and
    next() continues from wherever the seek left it, on or off the scan chain"""
    rng = np.random.default_rng({"restart": 11, "shared": 12, "bytes": 13}[kind])
    recs = corpus.random_records(rng, 3000, 1, 20, 0, 40)
    data, _ = _write(recs, 256, 2)             # many blocks: an index with many restart points
    seen_irregular = 0
    for t in range(6):
        bad = _corrupt_index(data, rng, kind)
        rd = _mods()
        try:
            r = rd.ReaderBuilder().verify_checksums(False).read(bad)
            seen_irregular += not r.index_regular()
        except (rd.MtblError, rd.ReferencePanic):
            pass
        for _ in range(5):
            keys = _probe_keys(rng, recs, 8)
            ops = []
            for _ in range(int(rng.integers(3, 10))):
                if rng.random() < 0.5:
                    ops.append(("seek", keys[int(rng.integers(0, len(keys)))]))
                else:
                    ops.append(int(rng.choice([1, 3, 20, 200])))
            mode = str(rng.choice(["iter", "from", "prefix", "range"]))
            k = keys[int(rng.integers(0, len(keys)))]
            _script_check(oracle, bad, False, mode, k if mode != "prefix" else k[:2], k + b"\x80", ops)
        for k in _probe_keys(rng, recs, 6):
            for mode, k1, k2 in (("from", k, b""), ("prefix", k[:2], b""), ("range", k, k + b"\xff")):
                try:
                    r = rd.ReaderBuilder().verify_checksums(False).read(bad)
                except (rd.MtblError, rd.ReferencePanic):
                    break
                exp = oracle.file_scan(bad, mode, k1, k2, verify=False)
                sc = {"from": lambda: r.iter_from(k1), "prefix": lambda: r.iter_prefix(k1),
                      "range": lambda: r.iter_range(k1, k2)}[mode]()
                if sc.end != exp["end"] or sc.records() != exp["records"]:
                    _dump_failure(bad, kind, mode, k1, k2)
                assert sc.end == exp["end"], (kind, mode, k1, k2, sc.nrec, len(exp["records"]), r.index_regular())
                assert sc.records() == exp["records"], (kind, mode, k1, k2)
    if kind != "bytes":
        assert seen_irregular > 0


def test_compressed_get_matches_oracle(oracle):
    rd = _mods()
    rng = np.random.default_rng(5)
    recs = corpus.random_records(rng, 2000, 1, 20, 0, 50)
    data, _ = _write(recs, 1024, 8, 2)
    r = rd.Reader(data)
    for k in _probe_keys(rng, recs, 40):
        exp = oracle.file_scan(data, "get", k)
        got = r.get(k)
        assert ([got] if got is not None else []) == [v for _, v in exp["records"]], k


def _long_key_records(rng, n=40):
    """keys of 66-200 KiB sharing long prefixes (entries carry shared of 60+ KiB), small values"""
    base = rng.integers(0, 256, 210_000, dtype=np.uint8).tobytes()
    keys = set()
    while len(keys) < n:
        kl = int(rng.integers(66_000, 200_000))
        p = int(rng.integers(60_000, kl))
        keys.add(base[:p] + rng.integers(0, 256, kl - p, dtype=np.uint8).tobytes())
    return [(k, bytes([i & 0xFF]) * int(rng.integers(0, 40))) for i, k in enumerate(sorted(keys))]


def test_keys_over_64kib(oracle):
    """keys longer than the emitting seek's 64 KiB LDS key (mtblx_block_seek_batch reports
    them; mtblx_block_seek_batch_kbuf carries the key in device memory): iter_from / prefix /
    range, the stateful iterator with seeks, Reader::get, and -- with a damaged index read with
    verification off -- the live index iterator over separators of 60+ KiB"""
    rd = _mods()
    rng = np.random.default_rng(64)
    recs = _long_key_records(rng)
    data, _ = _write(recs, 600_000, 2)          # several records per block, several blocks
    assert _bulk_check(oracle, data, True, rng, recs) > 0
    r = rd.Reader(data)
    for k in _probe_keys(rng, recs, 10):
        exp = oracle.file_scan(data, "get", k)
        got = r.get(k)
        assert got == (exp["records"][0][1] if exp["records"] and exp["records"][0][0] == k else None)
    for t in range(6):
        keys = _probe_keys(rng, recs, 6)
        ops = [("seek", keys[int(rng.integers(0, len(keys)))]) if rng.random() < 0.5 else int(rng.choice([1, 3, 30]))
               for _ in range(6)]
        _script_check(oracle, data, True, "from", keys[t % len(keys)], b"", ops)
    for kind in ("restart", "shared"):
        bad = _corrupt_index(data, rng, kind)
        keys = _probe_keys(rng, recs, 6)
        ops = [("seek", keys[1]), 3, ("seek", keys[2]), 5, ("seek", keys[0]), 40]
        _script_check(oracle, bad, False, "iter", b"", b"", ops)


def test_entry_offsets_zero_progress_entry():
    """r05: mtblx_entry_offsets' parallel pass walked each restart interval with no progress
    check, so an entry that does not advance (unterminated varints with non_shared = value_length
    = 0: the reference's next() yields it forever) spun one thread forever.  Such an interval is
    irregular now and the serial walk stops on the entry: offsets [0, 5], count 2, not regular."""
    _mods()
    import ctypes as C

    import torch
    from mtblx import _lib, codec
    blk = bytes.fromhex("0001014142" "8080808080" "00000000" "05000000" "02000000")
    d = torch.frombuffer(bytearray(blk), dtype=torch.uint8).to("cuda")
    offs = torch.full((16,), -1, dtype=torch.int64, device="cuda")
    cnt = torch.zeros(1, dtype=torch.int64, device="cuda")
    reg = torch.full((1,), 7, dtype=torch.int32, device="cuda")
    rc = _lib.lib().mtblx_entry_offsets(C.c_void_p(d.data_ptr()), len(blk), C.c_void_p(offs.data_ptr()), 16,
                                        C.c_void_p(cnt.data_ptr()), C.c_void_p(reg.data_ptr()),
                                        C.c_void_p(codec._stream_handle(None)))
    assert rc == 0
    assert int(cnt.item()) == 2 and int(reg.item()) == 0
    assert offs[:2].cpu().tolist() == [0, 5]
