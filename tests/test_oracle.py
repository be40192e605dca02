"""CPU tests: the oracle against the golden vectors and the reference's own test scenarios,
and the product's host layer (Writer, framing, CRC) against the oracle.  No GPU needed."""
import hashlib
import json
import os

import numpy as np
import pytest

import corpus

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def kat():
    return json.load(open(os.path.join(GOLD, "kat.json")))


# ---------------- oracle pinned by the golden vectors ----------------
def test_crc32c_check_value(oracle):
    assert oracle.crc32c(b"123456789") == 0xE3069283


def test_kat_one_key_file(oracle):
    k = kat()["one_key"]
    f = oracle.write_file([(b"hello", b"I'm the one")])
    assert len(f) == k["file_len"]
    assert f[:54].hex() == k["first_54"]
    assert hashlib.sha256(f).hexdigest() == k["sha256"]
    assert f == open(os.path.join(GOLD, "one_key.mtbl"), "rb").read()


def test_kat_empty_file(oracle):
    e = kat()["empty"]
    f = oracle.write_file([])
    assert len(f) == e["file_len"]
    assert hashlib.sha256(f).hexdigest() == e["sha256"]


def test_kat_block_contents(oracle):
    k = kat()["one_key"]
    st, recs = oracle.decode_block(bytes.fromhex(k["data_block_content"]))
    assert st == 0 and recs == [(b"hello", b"I'm the one")]
    st, recs = oracle.decode_block(bytes.fromhex(k["index_block_content"]))
    assert st == 0 and recs == [(b"hello", b"\x00")]
    assert oracle.crc32c(bytes.fromhex(k["data_block_content"])) == int(k["data_block_crc"], 16)


def test_restart_kat_hand_derived(oracle):
    """BlockBuilder's restart cadence (entries 0 / 16 / 32 restart with
    shared = 0, src/block_builder.rs:56-62), finish's three-entry restart array (:85-104), a
    2-byte non_shared varint and a 3-byte value_length varint (:69-73), pinned by the bytes
    tests/golden/make_golden.py assembles from hand-derived headers and offsets (no oracle)"""
    k = kat()["restart_kat"]
    import sys
    sys.path.insert(0, GOLD)
    import make_golden
    recs = make_golden.restart_kat_records()
    f = oracle.write_file(recs, k["block_size"], k["restart_interval"])
    assert len(f) == k["file_len"] and hashlib.sha256(f).hexdigest() == k["sha256"]
    assert f == open(os.path.join(GOLD, "restart_kat.mtbl"), "rb").read()
    assert f[:3].hex() == k["len_varint"] and f[3:7] == bytes.fromhex(k["data_block_crc"])[::-1]
    content = f[7: 7 + k["content_len"]]
    assert hashlib.sha256(content).hexdigest() == k["content_sha256"]
    n = int.from_bytes(content[-4:], "little")
    R = len(content) - 4 * (n + 1)
    assert [int.from_bytes(content[R + 4 * i: R + 4 * i + 4], "little") for i in range(n)] == k["restarts"]
    for i, hx in ((0, k["headers"]["restart"]), (16, k["headers"]["restart"]), (32, k["headers"]["restart"])):
        p = k["restarts"][i // 16]
        assert content[p: p + 3].hex() == hx
    st, got = oracle.decode_block(content)
    assert st == 0 and got == recs
    r = oracle.file_scan(f)
    assert r["end"] == oracle.END_NONE and r["records"] == recs and r["meta"] == k["metadata"]


@pytest.mark.parametrize("name,block,exp", corpus.quirk_blocks(), ids=[q[0] for q in corpus.quirk_blocks()])
def test_quirk_blocks_hand_derived(oracle, name, block, exp):
    st, recs = oracle.decode_block(block)
    assert st == exp["status"], exp["why"]
    assert recs == [(bytes.fromhex(a), bytes.fromhex(b)) for a, b in exp["records"]], exp["why"]


# ---------------- the reference's own tests, restated ----------------
def test_reference_writer_empty(oracle):
    """src/writer.rs:272-281 `empty`"""
    r = oracle.file_scan(oracle.write_file([]))
    assert r["end"] == oracle.END_NONE and r["records"] == []


def test_reference_writer_one_key(oracle):
    """src/writer.rs:283-298 `one_key`"""
    r = oracle.file_scan(oracle.write_file([(b"hello", b"I'm the one")]))
    assert len(r["records"]) == 1


def test_reference_separator_too_short(oracle):
    """src/writer.rs:300-305 `bytes_shortest_separator_to_short` must not panic"""
    assert oracle.shortest_separator(bytes([49, 115, 116]), bytes([50])) is not None


def test_varint_roundtrip_u32(oracle):
    """src/varint.rs:103-111 qc_codec_u32 (seeded sweep instead of quickcheck)"""
    rng = np.random.default_rng(7)
    vals = [0, 1, 127, 128, 16383, 16384, (1 << 21) - 1, 1 << 21, (1 << 28) - 1, 1 << 28, 2**32 - 1]
    vals += [int(x) for x in rng.integers(0, 2**32, 3000, dtype=np.uint64)]
    for v in vals:
        enc = oracle.varint_encode32(v)
        assert oracle.varint_decode32(enc) == (v, len(enc))


def test_varint_roundtrip_u64(oracle):
    """src/varint.rs:113-120 qc_codec_u64"""
    rng = np.random.default_rng(8)
    vals = [0, 1, 2**35, 2**56 - 1, 2**63, 2**64 - 1] + [int(x) for x in rng.integers(0, 2**63, 3000, dtype=np.uint64)]
    for v in vals:
        enc = oracle.varint_encode64(v)
        assert oracle.varint_decode64(enc) == (v, len(enc))


def test_varint_decode32_quirks(oracle):
    # unterminated within the 5-byte window: len 0, value = b0 & 0x7f (src/varint.rs:1-10,45-46)
    assert oracle.varint_decode32(bytes([0x85, 0x80, 0x80, 0x80, 0x80, 0x01])) == (5, 0)
    # 5th byte unmasked, high bits fall off the u32 (src/varint.rs:54)
    assert oracle.varint_decode32(bytes([0xFF, 0xFF, 0xFF, 0xFF, 0x7F])) == (0xFFFFFFFF, 5)
    # empty slice: the reference indexes data[0] -> panic
    assert oracle.varint_decode32(b"")[1] == -1


# ---------------- file-level iteration (examples/dump.rs, cfg1) ----------------
def test_cfg1_dump_roundtrip(oracle):
    from mtblx import synth
    recs = list(synth.cfg1_records())
    f = oracle.write_file(recs, block_size=4096)
    r = oracle.file_scan(f)
    assert r["end"] == oracle.END_NONE
    assert r["records"] == recs
    assert r["meta"][3] == len(recs) and r["meta"][1] == 4096


def test_get_prefix_range(oracle):
    recs = [(f"k{i:05}".encode(), f"v{i}".encode()) for i in range(0, 3000, 3)]
    f = oracle.write_file(recs, block_size=1024)
    assert oracle.file_scan(f, "get", b"k00300")["records"] == [(b"k00300", b"v300")]
    assert oracle.file_scan(f, "get", b"k00301")["records"] == []
    pre = oracle.file_scan(f, "prefix", b"k001")["records"]
    assert pre == [r for r in recs if r[0].startswith(b"k001")]
    rng = oracle.file_scan(f, "range", b"k00100", b"k00200")["records"]
    assert rng == [r for r in recs if b"k00100" <= r[0] <= b"k00200"]
    frm = oracle.file_scan(f, "from", b"k02990")["records"]
    assert frm == [r for r in recs if r[0] >= b"k02990"]


def test_crc_mismatch_panics(oracle):
    f = bytearray(oracle.write_file([(b"a", b"b"), (b"c", b"d")]))
    f[8] ^= 1  # inside the data block content
    assert oracle.file_scan(bytes(f))["end"] == oracle.END_PANIC
    assert oracle.file_scan(bytes(f), verify=False)["end"] != oracle.END_PANIC


def test_bad_magic_and_size(oracle):
    f = bytearray(oracle.write_file([(b"a", b"b")]))
    assert oracle.file_scan(bytes(f[:100]))["err"] == "InvalidMetadataSize"
    f[-1] ^= 0xFF
    assert oracle.file_scan(bytes(f))["err"] == "InvalidFormatVersion"


# ---------------- product host layer vs oracle ----------------
def test_product_writer_matches_oracle(oracle):
    import mtblx
    rng = np.random.default_rng(11)
    for trial in range(30):
        bs = int(rng.choice([1024, 1500, 4096, 8192]))
        iv = int(rng.choice([1, 4, 16, 33]))
        recs = corpus.random_records(rng, int(rng.integers(0, 400)), 0, 60, 0, 300)
        w = mtblx.WriterBuilder().block_size(bs).block_restart_interval(iv).memory()
        for k, v in recs:
            w.insert(k, v)
        assert w.into_inner() == oracle.write_file(recs, block_size=bs, restart_interval=iv), trial


def test_product_writer_out_of_order(oracle):
    import mtblx
    w = mtblx.Writer.memory()
    w.insert(b"b", b"1")
    with pytest.raises(mtblx.OutOfOrderKey):
        w.insert(b"a", b"2")


def test_product_crc32c_matches_oracle(oracle, mtblx_lib):
    import ctypes as C
    rng = np.random.default_rng(3)
    for n in [0, 1, 7, 8, 9, 63, 64, 1000, 4099]:
        a = rng.integers(0, 256, max(n, 1), dtype=np.uint8)
        got = mtblx_lib.mtblx_crc32c(a.ctypes.data_as(C.POINTER(C.c_uint8)), n)
        assert got == oracle.crc32c(a[:n].tobytes() if n else b"")


def test_product_block_dir(oracle):
    """the Writer's data-block directory points at exactly the framed contents"""
    import mtblx
    from mtblx import synth
    data, off, ln = synth.cfg2_file(50)
    raw = data.tobytes()
    r = oracle.file_scan(raw)
    assert r["end"] == oracle.END_NONE
    dec = oracle.decode_blocks(data, off, ln)
    assert (dec.status == 0).all() and int(dec.nrec.sum()) <= len(r["records"])
    flat = [rec for b in range(off.size) for rec in dec.records(b)]
    assert flat == r["records"][: len(flat)]


def test_iter_script_matches_file_scan_and_pins_seek_quirk(oracle):
    """oracle_iter_script (ReaderIntoIter with seek, src/reader.rs:219-405) agrees with
    oracle_file_scan for plain runs, and restates ReaderIntoIter::seek's block_offset quirk:
    block_offset starts at 0 and next() never updates it (:244-246, :269-271, :362-366), so
    seeking to a key of block 0 (offset 0) re-seeks the block the iterator currently holds."""
    recs = [(b"k%05d" % i, b"v%d" % i) for i in range(3000)]
    f = oracle.write_file(recs, 512, 4)
    for mode, k, k2 in [("iter", b"", b""), ("from", b"k00100", b""), ("prefix", b"k001", b""),
                        ("range", b"k00500", b"k00700"), ("get", b"k00300", b"")]:
        a = oracle.file_scan(f, mode, k, k2)
        b = oracle.iter_script(f, mode, k, k2, [10 ** 9])
        assert a["records"] == b["records"] and a["end"] == b["end"]
    r = oracle.iter_script(f, "from", b"k01000", b"", [3, ("seek", b"k00002"), 2, ("seek", b"k02999"), 5,
                                                       ("seek", b"zzz"), 3])
    got = [k for k, _ in r["records"]]
    # k00002 lives in block 0: no reload, the held block (first key k00978) is re-seeked
    assert got[:3] == [b"k01000", b"k01001", b"k01002"]
    assert got[3:5] == [b"k00978", b"k00979"]
    assert got[5:] == [b"k02999"]
    assert r["ops"] == [(3, 0), (0, 0), (2, 0), (0, 0), (1, 1), (0, 0), (0, 1)]
    # a seek whose block offset differs reloads: from an iterator built by into_iter.  The block
    # is seeked to the landed separator (src/reader.rs:305,328): these separators equal their
    # block's last key ('9'+1 == ':' leaves no shorter separator), so next() yields that key
    r2 = oracle.iter_script(f, "iter", b"", b"", [2, ("seek", b"k02000"), 2])
    got2 = [k for k, _ in r2["records"]]
    seps = [k for k, _ in oracle.index_records(f)]
    assert got2[:2] == [b"k00000", b"k00001"]
    assert got2[2] == min(x for x in seps if x >= b"k02000") and got2[3] > got2[2]


def test_seek_kat_hand_derived(oracle):
    """ReaderIntoIter::seek against the hand-derived vectors of tests/golden/kat.json (seek_kat):
    the data block is seeked to the landed index entry's separator, covering a separator equal
    to the block's last key, a bumped one and a write_u16-appended one"""
    kat = json.load(open(os.path.join(GOLD, "kat.json")))["seek_kat"]
    recs = [(k.encode(), bytes([0x41 + i]) * kat["value_len"]) for i, k in enumerate(kat["keys"])]
    f = oracle.write_file(recs, kat["block_size"], kat["restart_interval"])
    assert [k.decode() for k, _ in oracle.index_records(f)] == kat["separators"]
    vals = dict(recs)
    for sc in kat["scripts"]:
        ops = [o if isinstance(o, int) else ("seek", o[1].encode()) for o in sc["ops"]]
        r = oracle.iter_script(f, sc["mode"], sc["key"].encode(), b"", ops)
        assert r["end"] == 0
        assert [k.decode() for k, _ in r["records"]] == sc["yields"], sc["why"]
        assert all(v == vals[k] for k, v in r["records"])
