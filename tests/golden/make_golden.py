"""Generate / verify the golden fixtures under tests/golden/.

1. kat.json: known-answer vectors HAND-DERIVED in SURVEY.md §2.2 from the reference's
   src/writer.rs, src/block_builder.rs, src/metadata.rs (the reference publishes no
   fixtures and cannot be built here).  They pin the reference tests `one_key` and
   `empty` (src/writer.rs:272-298) byte-exactly.
2. one_key.mtbl / empty.mtbl: the files those vectors describe, written by the oracle
   and checked against kat.json before being (re)written.
3. one_key_v1.mtbl / empty_v1.mtbl: the same two files in FormatV1, which the reference reads
   (src/metadata.rs:29-33: magic 0x77846676; src/reader.rs:54-56,146-148: u32 LE block
   lengths instead of varint64) but never writes (src/writer.rs:215).  Their bytes are
   assembled here from the hand-derived pieces in KAT["one_key_v1"] / KAT["empty_v1"] and must
   equal what tests/corpus.py:to_v1 makes of the V2 files.
4. quirk_blocks.json: hand-constructed single blocks with the outcome derived by hand
   from src/block.rs (status + records) — pins the oracle's panic / None / loop /
   Vec-capacity semantics independently of its code.

Usage:  python tests/golden/make_golden.py [--check]
"""
import hashlib
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "oracle"))

# --- SURVEY.md §2.2 (hand derivation) ---
KAT = {
    "crc32c_check": {"input": "123456789", "crc": "e3069283"},
    "one_key": {
        "insert": [["hello", "I'm the one"]],
        "data_block_content": "00050b68656c6c6f49276d20746865206f6e650000000001000000",
        "data_block_crc": "3f400b02",
        "index_block_content": "00050168656c6c6f000000000001000000",
        "index_block_crc": "deec1759",
        "file_len": 566,
        "metadata": [32, 8192, 0, 1, 1, 32, 22, 5, 11],
        "first_54": "1b020b403f00050b68656c6c6f49276d20746865206f6e650000000001000000115917ecde00050168656c6c6f000000000001000000",
        "sha256": "ba687784368babc7a8bf12033fafd36091e0c05eaa28c5838bace82a023b26b7",
    },
    # FormatV1 (hand-derived): u32 LE content lengths, the same checksums and contents; the
    # index value varint64(0) and the footer offsets move with the 3 extra framing bytes per block
    "one_key_v1": {
        "data_frame": "1b000000" "020b403f" "00050b68656c6c6f49276d20746865206f6e650000000001000000",
        "index_frame": "11000000" "5917ecde" "00050168656c6c6f000000000001000000",
        "file_len": 572,
        "metadata": [35, 8192, 0, 1, 1, 35, 25, 5, 11],
        "magic": "76668477",
        "sha256": "c8dec613b1bb3032acc16fa0e7f38f0480da6976f70699d41ed18cfaa7b32c8f",
        "records": [["hello", "I'm the one"]],
    },
    "empty_v1": {
        "index_frame": "08000000" "32186d51" "0000000001000000",
        "file_len": 528,
        "metadata": [0, 8192, 0, 0, 0, 0, 16, 0, 0],
        "magic": "76668477",
        "records": [],
    },
    "empty": {
        "index_block_content": "0000000001000000",
        "index_block_crc": "516d1832",
        "file_len": 525,
        "metadata": [0, 8192, 0, 0, 0, 0, 13, 0, 0],
        "sha256": "d19adf5e336a2b4b6e92c178a3e919026ee4f6899e161367af361fdcf9935435",
    },
}

# --- hand-derived single-block outcomes (src/block.rs; release-mode arithmetic) ---
# status: 0 OK, 1 INVALID_BLOCK (Block::init None), 2 CORRUPT (panic), 3 LOOP (never terminates)
QUIRKS = [
    {"name": "len3_invalid", "block": "000000", "status": 1, "records": [],
     "why": "len < 4 -> Block::init None (block.rs:19-20)"},
    {"name": "len6_corrupt", "block": "000000000000", "status": 2, "records": [],
     "why": "len in [4,8): num_restarts assert (block.rs:59)"},
    {"name": "zero_restarts", "block": "0000000000000000", "status": 2, "records": [],
     "why": "n == 0 passes Block::init, BlockIter::init asserts n > 0 (block.rs:79)"},
    {"name": "too_many_restarts", "block": "0000000005000000", "status": 1, "records": [],
     "why": "4*(n+1) > len wraps (release) -> 64-bit branch wraps -> > len-4 -> None"},
    {"name": "empty_block", "block": "0000000001000000", "status": 0, "records": [],
     "why": "restart[0] = 0 = restart_offset -> no entries"},
    {"name": "one_entry", "block": "000101414200000000" "01000000", "status": 0, "records": [["41", "42"]],
     "why": "fast-path header (0,1,1)"},
    {"name": "first_shared_nonzero", "block": "010101414200000000" "01000000", "status": 2, "records": [],
     "why": "fresh key Vec has capacity 0 < shared=1: assert (block.rs:132)"},
    {"name": "vec_capacity_quirk", "block": "0002006162" "05010063" "090000" "00000000" "01000000", "status": 2,
     "records": [["6162", ""], ["616263", ""]],
     "why": "e1 shared=5 > len 2 but <= capacity 8: truncate no-op -> 'abc'; e2 shared=9 > capacity 8 -> panic"},
    {"name": "unterminated_loop", "block": "8080808080" "00000000" "01000000", "status": 3, "records": [["", ""]],
     "why": "5 continuation bytes: varint len 0, cursor never advances, next == current forever"},
    {"name": "noncanonical_varints", "block": "8000810080" "0041" "00000000" "01000000", "status": 0,
     "records": [["41", ""]], "why": "slow path: shared=0 (80 00), non_shared=1 (81 00), value_length=0 (80 00)"},
    {"name": "restart0_not_zero", "block": "0001014142" "0001014344" "05000000" "01000000", "status": 0,
     "records": [["43", "44"]], "why": "the scan starts at restart_point(0) = 5, skipping the first entry"},
    {"name": "restart0_at_end", "block": "0001014142" "05000000" "01000000", "status": 0, "records": [],
     "why": "restart_point(0) >= restart_offset -> iterator invalid at once"},
    {"name": "header_truncated", "block": "0001" "00000000" "01000000", "status": 2, "records": [],
     "why": "limit - p = 2 < 3 -> decode_entry Err -> unwrap panic (block.rs:217-219,131)"},
    {"name": "entry_overruns", "block": "00050041" "00000000" "01000000", "status": 2, "records": [],
     "why": "non_shared + value_length = 5 > limit - p = 1 (block.rs:235)"},
    {"name": "u32_sum_overflow", "block": "00" "8080808008" "8080808008" "00000000" "01000000", "status": 2,
     "records": [], "why": "non_shared = value_length = 2^31: u32 sum overflows; the record is never yielded"},
    {"name": "second_entry_corrupt", "block": "0001014142" "00050043" "00000000" "01000000", "status": 2,
     "records": [["41", "42"]], "why": "first record yielded, second overruns limit -> panic"},
]


# --- ReaderIntoIter::seek (src/reader.rs:302-335), hand-derived ---
# Writer(block_size 1024, restart interval 16, None); every value is 300 bytes, so the flush
# rule (src/writer.rs:125-130) cuts a block after three 8-byte keys (311 + 304 + 304 B).
# Separators (src/writer.rs:239-265):
#   block 0 key-0000 .. key-0002 | next key-0003: '2'+1 == '3', no u16 room -> "key-0002" (= last key)
#   block 1 key-0003 .. key-0005 | next key-0007: '5'+1 <  '7'              -> "key-0006" (bumped)
#   block 2 key-0007, key-0008, key-0009ab | next key-000:ac: '9'+1 == ':', diff 7 < 10-2 ->
#           write_u16 APPENDS BE16("9a")+1 = "9b"                           -> "key-0009ab9b"
#   block 3 key-000:ac, key-000;  (last index entry = the last key, :158-162)
# seek(k) lands the index iterator on the first separator >= k and seeks the data block to
# that SEPARATOR (`key` is shadowed at :305), so seek + next() yields the landed block's last
# record when the separator equals it, else the next block's first record.
SEEK_KAT = {
    "block_size": 1024, "restart_interval": 16, "value_len": 300,
    "keys": ["key-0000", "key-0001", "key-0002", "key-0003", "key-0004", "key-0005", "key-0007", "key-0008",
             "key-0009ab", "key-000:ac", "key-000;"],
    "separators": ["key-0002", "key-0006", "key-0009ab9b", "key-000;"],
    "scripts": [
        {"mode": "iter", "key": "", "ops": [["seek", "key-0001"], 3],
         "yields": ["key-0002", "key-0003", "key-0004"],
         "why": "index entry 0 (sep key-0002 = last key), block 0 already held (offset 0): seek(key-0002)"},
        {"mode": "iter", "key": "", "ops": [["seek", "key-0004"], 2], "yields": ["key-0007", "key-0008"],
         "why": "entry 1, sep key-0006 past block 1's keys: next() moves to block 2"},
        {"mode": "iter", "key": "", "ops": [["seek", "key-0008"], 1], "yields": ["key-000:ac"],
         "why": "entry 2, appended sep key-0009ab9b > key-0009ab: next() moves to block 3"},
        {"mode": "iter", "key": "", "ops": [["seek", "key-000;"], 2], "yields": ["key-000;"],
         "why": "last entry: the last record, then None"},
        {"mode": "iter", "key": "", "ops": [["seek", "key-000<"], 1], "yields": [],
         "why": "past the last separator: valid = false"},
        {"mode": "from", "key": "key-0005", "ops": [3, ["seek", "key-0000"], 4],
         "yields": ["key-0005", "key-0007", "key-0008", "key-0007", "key-0008", "key-0009ab", "key-0003"],
         "why": "new_from seeks block 1 with the CALLER's key; seek(key-0000) lands entry 0 at offset 0 = "
                "block_offset: the held block 2 is seeked to key-0002 -> key-0007; after block 2 the index "
                "iterator (at entry 0) moves to entry 1 -> block 1"},
    ],
}


# --- BlockBuilder's restart cadence and multi-byte varint headers, hand-derived ---
# One data block of 33 records at restart interval 16 (src/block_builder.rs:49-83): entries 0, 16
# and 32 start a restart (counter == interval -> push buf.len(), counter = 0, shared = 0,
# :56-62); every other entry shares the 4-byte prefix "kat-" with its predecessor.
#   key_i   = "kat-" + chr(0x41 + i)            (5 B; 'A' .. 'a')
#   key_20  = "kat-U" + "x" * 130               (135 B: non_shared 131 -> 2-byte varint 83 01)
#   value_i = chr(0x30 + i % 10) * (i % 4)      (0..3 B)
#   value_10 = 0xa5 * 16500                     (value_length 16500 -> 3-byte varint f4 80 01)
# Entry sizes (header + non_shared + value_length):
#   restart entries 0, 16, 32: header 00 05 00, 5 key bytes, no value    -> 8
#   entry i (other):           header 04 01 0v, 1 key byte, v = i % 4     -> 4 + i % 4
#   entry 10:                  header 04 01 f4 80 01, 1 key byte, 16500 B -> 16506
#   entry 20:                  header 04 83 01 00, 131 key bytes         -> 135
#   restart[1] = 8 + (5+6+7+4+5+6+7+4+5 +7+4+5+6+7 = 78) + 16506          = 16592
#   restart[2] = 16592 + 8 + (5+6+7 +5+6+7+4+5+6+7+4+5+6+7 = 80) + 135     = 16815
#   buf = 16815 + 8 = 16823; finish (:85-104): u32 LE 0, 16592, 16815 and n = 3 -> L = 16839
# write_block (src/writer.rs:203-237): varint64(16839) = c7 83 01 (16384 + 3*128 + 71), crc32c,
# content -> 3 + 4 + 16839 = 16846 B.  Writer::into_inner: one index entry, key = the last key
# "kat-a" (no separator: nothing follows, :158-162), value varint64(0) = 00 ->
# content 000501 6b61742d61 00 | 00000000 | 01000000 (17 B), frame 11 + crc + content = 22 B.
# Footer (src/metadata.rs:61-79): {16846, 65536, 0, 33, 1, 16846, 22, 295, 16546}, magic at 508.
# bytes_keys = 32 * 5 + 135 = 295; bytes_values = sum(i % 4, i != 10) + 16500 = 46 + 16500.
RESTART_KAT = {
    "block_size": 65536, "restart_interval": 16, "n": 33,
    "headers": {"restart": "000500", "regular": "0401", "e10": "0401f48001", "e20": "04830100"},
    "restarts": [0, 16592, 16815],
    "content_len": 16839,
    "len_varint": "c78301",
    "data_frame_len": 16846,
    "index_block_content": "0005016b61742d61000000000001000000",
    "file_len": 17380,
    "metadata": [16846, 65536, 0, 33, 1, 16846, 22, 295, 16546],
    # computed from the bytes above by this file's own bitwise CRC-32C / hashlib (restart_kat_bytes)
    "data_block_crc": "3b89ccac",
    "index_block_crc": "64ce6dc3",
    "content_sha256": "db586532e85ed44fa77874c1d369a35daba9ef12fc795f16fef6d9255d7f9792",
    "sha256": "12ed53a371c51f15a4a8a3876251b27790de6d38683816ab2bf9ec2a555119ec",
}


def restart_kat_records():
    recs = []
    for i in range(33):
        k = b"kat-" + bytes([0x41 + i]) + (b"x" * 130 if i == 20 else b"")
        v = b"\xa5" * 16500 if i == 10 else bytes([0x30 + i % 10]) * (i % 4)
        recs.append((k, v))
    return recs


def crc32c_bitwise(b: bytes) -> int:
    """CRC-32C (Castagnoli, reflected 0x82F63B78, init / xorout 0xFFFFFFFF), bit by bit"""
    c = 0xFFFFFFFF
    for x in b:
        c ^= x
        for _ in range(8):
            c = (c >> 1) ^ (0x82F63B78 if c & 1 else 0)
    return c ^ 0xFFFFFFFF


def restart_kat_bytes():
    """assemble the RESTART_KAT block and file from the hand-derived pieces (no oracle)"""
    k = RESTART_KAT
    h = k["headers"]
    buf = b""
    starts = []
    for i, (key, val) in enumerate(restart_kat_records()):
        starts.append(len(buf))
        if i % 16 == 0:
            buf += bytes.fromhex(h["restart"]) + key
        elif i == 10:
            buf += bytes.fromhex(h["e10"]) + key[4:] + val
        elif i == 20:
            buf += bytes.fromhex(h["e20"]) + key[4:] + val
        else:
            buf += bytes.fromhex(h["regular"]) + bytes([i % 4]) + key[4:] + val
    assert [starts[0], starts[16], starts[32]] == k["restarts"]
    content = buf + b"".join(r.to_bytes(4, "little") for r in k["restarts"]) + (3).to_bytes(4, "little")
    assert len(content) == k["content_len"]
    crc = crc32c_bitwise(content)
    frame = bytes.fromhex(k["len_varint"]) + crc.to_bytes(4, "little") + content
    assert len(frame) == k["data_frame_len"]
    idx = bytes.fromhex(k["index_block_content"])
    icrc = crc32c_bitwise(idx)
    footer = b"".join(m.to_bytes(8, "little") for m in k["metadata"])
    f = frame + bytes([len(idx)]) + icrc.to_bytes(4, "little") + idx + footer + b"\0" * (508 - len(footer)) + \
        (0x4D54424C).to_bytes(4, "little")
    assert len(f) == k["file_len"]
    return content, crc, idx, icrc, f


def check_restart_kat():
    """the hand-assembled bytes carry the recorded checksums / digests, and the oracle Writer and
    block decoder agree with them"""
    import pyoracle as o
    k = RESTART_KAT
    assert crc32c_bitwise(b"123456789") == int(KAT["crc32c_check"]["crc"], 16)
    content, crc, idx, icrc, f = restart_kat_bytes()
    assert f"{crc:08x}" == k["data_block_crc"] and f"{icrc:08x}" == k["index_block_crc"], (hex(crc), hex(icrc))
    assert hashlib.sha256(content).hexdigest() == k["content_sha256"]
    assert hashlib.sha256(f).hexdigest() == k["sha256"]
    recs = restart_kat_records()
    assert o.write_file(recs, k["block_size"], k["restart_interval"]) == f
    st, got = o.decode_block(content)
    assert st == 0 and got == recs
    return f


def seek_kat_records():
    v = SEEK_KAT["value_len"]
    return [(k.encode(), bytes([0x41 + i]) * v) for i, k in enumerate(SEEK_KAT["keys"])]


def seek_kat_ops(script):
    return [o if isinstance(o, int) else ("seek", o[1].encode()) for o in script["ops"]]


def build_files():
    import pyoracle as o
    one = o.write_file([(b"hello", b"I'm the one")])
    empty = o.write_file([])
    return one, empty


def v1_kat_bytes(name):
    """a FormatV1 KAT file from its hand-derived pieces: frames, zero-padded footer, magic"""
    k = KAT[name]
    body = bytes.fromhex(k.get("data_frame", "") + k["index_frame"])
    footer = b"".join(m.to_bytes(8, "little") for m in k["metadata"])
    return body + footer + b"\0" * (508 - len(footer)) + bytes.fromhex(k["magic"])


def check_v1(one, empty):
    """the V1 KATs: hand bytes == corpus.to_v1(V2 file); the oracle reads them back"""
    import pyoracle as o
    sys.path.insert(0, os.path.dirname(HERE))
    import corpus
    for name, v2 in (("one_key_v1", one), ("empty_v1", empty)):
        k = KAT[name]
        b = v1_kat_bytes(name)
        assert len(b) == k["file_len"], (name, len(b))
        if "sha256" in k:
            assert hashlib.sha256(b).hexdigest() == k["sha256"]
        assert corpus.to_v1(v2) == b, name
        r = o.file_scan(b)
        assert r["version"] == 0 and r["end"] == 0 and r["meta"] == k["metadata"], (name, r)
        assert r["records"] == [(a.encode(), v.encode()) for a, v in k["records"]], (name, r["records"])
    return v1_kat_bytes("one_key_v1"), v1_kat_bytes("empty_v1")


def check(one, empty):
    import pyoracle as o
    assert o.crc32c(b"123456789") == int(KAT["crc32c_check"]["crc"], 16)
    k = KAT["one_key"]
    assert len(one) == k["file_len"]
    assert one[:54].hex() == k["first_54"]
    assert hashlib.sha256(one).hexdigest() == k["sha256"]
    assert o.crc32c(bytes.fromhex(k["data_block_content"])) == int(k["data_block_crc"], 16)
    assert o.crc32c(bytes.fromhex(k["index_block_content"])) == int(k["index_block_crc"], 16)
    e = KAT["empty"]
    assert len(empty) == e["file_len"]
    assert hashlib.sha256(empty).hexdigest() == e["sha256"]
    assert o.crc32c(bytes.fromhex(e["index_block_content"])) == int(e["index_block_crc"], 16)


def main():
    one, empty = build_files()
    check(one, empty)
    one1, empty1 = check_v1(one, empty)
    rk = check_restart_kat()
    if "--check" in sys.argv:
        assert open(os.path.join(HERE, "restart_kat.mtbl"), "rb").read() == rk
        assert open(os.path.join(HERE, "one_key.mtbl"), "rb").read() == one
        assert open(os.path.join(HERE, "empty.mtbl"), "rb").read() == empty
        assert open(os.path.join(HERE, "one_key_v1.mtbl"), "rb").read() == one1
        assert open(os.path.join(HERE, "empty_v1.mtbl"), "rb").read() == empty1
        print("golden fixtures OK")
        return
    open(os.path.join(HERE, "one_key.mtbl"), "wb").write(one)
    open(os.path.join(HERE, "empty.mtbl"), "wb").write(empty)
    open(os.path.join(HERE, "one_key_v1.mtbl"), "wb").write(one1)
    open(os.path.join(HERE, "empty_v1.mtbl"), "wb").write(empty1)
    open(os.path.join(HERE, "restart_kat.mtbl"), "wb").write(rk)
    json.dump(dict(KAT, seek_kat=SEEK_KAT, restart_kat=RESTART_KAT), open(os.path.join(HERE, "kat.json"), "w"), indent=1)
    json.dump(QUIRKS, open(os.path.join(HERE, "quirk_blocks.json"), "w"), indent=1)
    print("wrote tests/golden/{one_key,empty}{,_v1}.mtbl, kat.json, quirk_blocks.json")


if __name__ == "__main__":
    main()
