"""Device Writer end to end: plan (flush rule) + encode_blocks (BlockBuilder,
write_block framing) + mtblx_encode_index (index block with bytes_shortest_separator's write_u16
APPEND quirk, index write_block, 512-byte footer) -> a whole .mtbl file on the GPU, byte-identical
to the oracle Writer (src/writer.rs restated), which the golden files pin; then read back by the
device Reader."""
import os

import numpy as np
import pytest

import corpus

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _dev():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from mtblx import encode
    return encode


def _device_file(records, bs, iv):
    encode = _dev()
    recs = encode.DeviceRecords.from_list(records)
    return encode.write_file(recs, bs, iv).cpu().numpy().tobytes()


def test_golden_files():
    """src/writer.rs:272-298 `empty` and `one_key` (SURVEY §2.2 KATs)."""
    assert _device_file([], 8192, 16) == open(os.path.join(GOLD, "empty.mtbl"), "rb").read()
    assert _device_file([(b"hello", b"I'm the one")], 8192, 16) == open(os.path.join(GOLD, "one_key.mtbl"), "rb").read()


def test_restart_kat_device():
    """the hand-derived restart-cadence / multi-byte-header KAT
    (tests/golden/make_golden.py RESTART_KAT: 33 records at interval 16 -> restarts at entries
    0 / 16 / 32, a 2-byte non_shared varint, a 3-byte value_length varint) -- written by the
    device Writer (k_plan + k_encode + the index kernels), encoded unframed by k_encode, and
    decoded by the device (mtblx_decode_blocks, verified and fused-verified, and the Reader)"""
    encode = _dev()
    import json
    import sys

    import torch
    from mtblx import codec, reader
    sys.path.insert(0, GOLD)
    import make_golden
    k = json.load(open(os.path.join(GOLD, "kat.json")))["restart_kat"]
    gold = open(os.path.join(GOLD, "restart_kat.mtbl"), "rb").read()
    recs = make_golden.restart_kat_records()
    assert _device_file(recs, k["block_size"], k["restart_interval"]) == gold
    d = encode.DeviceRecords.from_list(recs)
    blk = torch.tensor([0, len(recs)], dtype=torch.int64, device="cuda")
    e = encode.encode_blocks(d, blk, k["restart_interval"], framed=False)
    content = gold[7: 7 + k["content_len"]]
    o, n = int(e.blk_off[0].item()), int(e.blk_len[0].item())
    assert e.out.cpu().numpy()[o: o + n].tobytes() == content
    f = np.frombuffer(gold, np.uint8)
    batch = codec.DeviceBatch.from_host(f, np.array([7], np.uint64), np.array([k["content_len"]], np.uint32))
    h = codec.decode_blocks(batch).to_host()
    assert int(h.status[0]) == 0 and h.records(0) == recs
    for fused in (False, True):
        out, crc, bad = codec.decode_verify(batch, framed=True, fused=fused)
        torch.cuda.synchronize()
        assert out.to_host().records(0) == recs
        assert int(crc.cpu().numpy().view(np.uint32)[0]) == int(k["data_block_crc"], 16) and int(bad[0].item()) == 0
    assert reader.Reader(f).iter().records() == recs


def _append_quirk_records(n, vlen):
    """consecutive pairs (.. j, 0xFF ..) < (.. j+1, 0x00 ..): every block boundary between
    them takes the separator's write_u16 APPEND branch (src/writer.rs:254-262)"""
    recs = []
    for j in range(n):
        hi = j.to_bytes(2, "big")
        recs.append((b"k" + hi + b"\xff\x01\x01", bytes([j % 251]) * (vlen + (j * 7) % 50)))
        recs.append((b"k" + (j + 1).to_bytes(2, "big") + b"\x00\x00\x00", bytes([j % 241]) * ((j * 13) % 40)))
    return recs


@pytest.mark.parametrize("bs,iv", [(1024, 16), (4096, 16), (8192, 1), (4096, 3), (65536, 16), (2000, 40)])
def test_random_files_byte_identical(oracle, bs, iv):
    rng = np.random.default_rng(bs + iv)
    recs = corpus.random_records(rng, 3000, 0, 60, 0, 300)
    dev = _device_file(recs, bs, iv)
    assert dev == oracle.write_file(recs, bs, iv)


def test_separator_append_quirk(oracle):
    recs = _append_quirk_records(1500, 37)
    for bs in (1024, 1500, 4096):
        dev = _device_file(recs, bs, 16)
        exp = oracle.write_file(recs, bs, 16)
        assert dev == exp
    # the quirk is really exercised: some index key is a data key + 2 appended bytes
    from mtblx import reader
    r = reader.Reader(np.frombuffer(dev, np.uint8))
    keys = set(k for k, _ in recs)
    h = r.index.to_host()
    ikeys = [k for k, _ in h.records(0)]
    assert any(len(k) == 8 and k[:6] in keys for k in ikeys)


def test_cfg3_scheme_file_roundtrip(oracle):
    """Zipf 8..256 B keys (cfg3's scheme), 64 KiB blocks: byte-identical to the oracle Writer,
    and the device Reader yields exactly the records."""
    _dev()
    import torch
    from mtblx import reader, synth
    from mtblx.encode import write_file
    recs_d, _ = synth.cfg3_records_device(20000, seed=synth.SEED_CFG3 + 77)
    f = write_file(recs_d, 65536, 16)
    ke = recs_d.key_end.cpu().numpy()
    ve = recs_d.val_end.cpu().numpy()
    kb = recs_d.keys.cpu().numpy().tobytes()
    vb = recs_d.vals.cpu().numpy().tobytes()
    recs = [(kb[(ke[i - 1] if i else 0): ke[i]], vb[(ve[i - 1] if i else 0): ve[i]]) for i in range(ke.size)]
    assert f.cpu().numpy().tobytes() == oracle.write_file(recs, 65536, 16)
    s = reader.Reader(f).iter()
    torch.cuda.synchronize()
    assert s.end == reader.END_NONE and s.nrec == len(recs)
    assert s.records() == recs
