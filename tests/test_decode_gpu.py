"""GPU parity: the HIP decoder (through the C ABI) vs the CPU oracle, bit-exact.

All cases run in ONE process.  The full BASELINE cfg2 size (100 000 blocks) is compared with the
oracle block for block (the oracle decodes it in ~0.3 s) and also checked through size-independent
properties (decode(encode(x)) == x against the generator's own records, totals == footer counts).
"""
import numpy as np
import pytest

import corpus

pytestmark = pytest.mark.gpu


def _dev():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from mtblx import codec
    return codec


def device_decode(data, off, ln):
    codec = _dev()
    batch = codec.DeviceBatch.from_host(data, off, ln)
    out = codec.decode_blocks(batch)
    import torch
    torch.cuda.synchronize()
    return out.to_host()


def assert_same(dev, orc, nblk):
    assert np.array_equal(dev.status, orc.status), np.nonzero(dev.status != orc.status)[0][:10]
    assert np.array_equal(dev.nrec, orc.nrec), np.nonzero(dev.nrec != orc.nrec)[0][:10]
    assert np.array_equal(dev.rec_base, orc.rec_base)
    assert np.array_equal(dev.key_base, orc.key_base)
    assert np.array_equal(dev.val_base, orc.val_base)
    nr = int(orc.nrec.sum())
    assert dev.totals[0] == nr and dev.totals[1] == orc.keys.size and dev.totals[2] == orc.vals.size
    assert dev.totals[3] == 0
    assert np.array_equal(dev.key_end, orc.key_end)
    assert np.array_equal(dev.val_end, orc.val_end)
    if not np.array_equal(dev.keys, orc.keys):
        bad = np.nonzero(dev.keys != orc.keys)[0]
        raise AssertionError(f"key bytes differ at {bad[:10]} (of {bad.size})")
    assert np.array_equal(dev.vals, orc.vals)


def run_both(oracle, blocks, rng=None, lead=0):
    data, off, ln = corpus.pack(blocks, lead=lead, rng=rng)
    orc = oracle.decode_blocks(data, off, ln)
    dev = device_decode(data, off, ln)
    assert_same(dev, orc, len(blocks))
    return orc


def test_quirk_blocks(oracle):
    q = corpus.quirk_blocks()
    orc = run_both(oracle, [b for _, b, _ in q])
    for i, (_, _, exp) in enumerate(q):
        assert orc.status[i] == exp["status"]


def test_builder_blocks_all_shapes(oracle):
    blocks = corpus.builder_blocks(oracle, seed=5, count=300, max_bytes=8100)
    orc = run_both(oracle, blocks, rng=np.random.default_rng(1), lead=3)
    assert (orc.status == 0).all()


def test_mutated_blocks(oracle):
    blocks = corpus.mutated_blocks(oracle, seed=9, count=800)
    orc = run_both(oracle, blocks, rng=np.random.default_rng(2))
    # the corpus must exercise every outcome
    assert {0, 1, 2} <= set(orc.status.tolist())


def test_large_blocks_generic_path(oracle):
    rng = np.random.default_rng(4)
    blocks = []
    for n in (200, 400, 900):
        recs = corpus.random_records(rng, n, 4, 60, 10, 120)
        blocks.append(oracle.build_block(recs))
    assert max(len(b) for b in blocks) > 8192
    run_both(oracle, blocks + corpus.builder_blocks(oracle, seed=6, count=20))


def test_block_at_end_of_buffer(oracle):
    """last block ends exactly at data_len: staging must not read past the buffer"""
    blocks = corpus.builder_blocks(oracle, seed=12, count=7, max_bytes=4000)
    for lead in (0, 1, 5, 15):
        run_both(oracle, blocks, lead=lead)


def test_cfg2_sample_vs_oracle(oracle):
    from mtblx import synth
    data, off, ln = synth.cfg2_file(3000)
    orc = oracle.decode_blocks(data, off, ln)
    dev = device_decode(data, off, ln)
    assert_same(dev, orc, off.size)


def test_overflow_reported(oracle):
    codec = _dev()
    import torch
    from mtblx import synth
    data, off, ln = synth.cfg2_file(64)
    batch = codec.DeviceBatch.from_host(data, off, ln)
    orc = oracle.decode_blocks(data, off, ln)
    out = codec.DecodedBlocks(off.size, int(orc.nrec.sum()), orc.keys.size // 2, orc.vals.size)
    ws = codec.Workspace(off.size)
    codec.decode_into(batch, out, ws)
    torch.cuda.synchronize()
    h = out.to_host()
    assert h.totals[3] & 1
    st = h.status
    assert (st[: off.size // 2 - 1] == 0).all() and (st[off.size // 2 + 1:] == 5).all()


def test_cfg2_full_vs_oracle(oracle):
    """BASELINE cfg2 at full size (100 000 x 4 KiB blocks): every block's status, record count,
    bases, key / value END offsets and every key and value byte equal to the oracle's decode of
    the same blocks (src/block.rs:119-238 restated, oracle/mtbl_oracle.c)."""
    from mtblx import synth
    data, off, ln = synth.cfg2_file(100_000)
    orc = oracle.decode_blocks(data, off, ln)
    assert (orc.status == 0).all() and int(orc.nrec.sum()) == 5_100_000
    dev = device_decode(data, off, ln)
    assert_same(dev, orc, off.size)


def test_cfg2_full_roundtrip_property():
    """BASELINE cfg2 at full size (100 k blocks): decode(encode(x)) == x for every record."""
    codec = _dev()
    import torch
    from mtblx import synth
    nblk = 100_000
    data, off, ln = synth.cfg2_file(nblk)
    batch = codec.DeviceBatch.from_host(data, off, ln)
    out = codec.decode_blocks(batch)
    torch.cuda.synchronize()
    nr, kb, vb, flags = out.totals_host()
    assert flags == 0
    assert (out.status[:nblk] == 0).all().item()
    kl, vl = 16, 64
    # regenerate the writer's input records (same generator call as synth.cfg2_file)
    dk = out.keys[:kb].cpu().numpy()
    dv = out.vals[:vb].cpu().numpy()
    assert kb == nr * kl and vb == nr * vl
    big_keys, big_vals, _, _ = synth.cfg2_arrays(int(nblk * ((4096 - 64) // 79) * 1.02) + 64)
    assert np.array_equal(dk, big_keys[: kb])
    assert np.array_equal(dv, big_vals[: vb])
    ke = out.key_end[:nr].cpu().numpy().view(np.uint32)
    nrec = out.nrec[:nblk].cpu().numpy()
    rb = np.concatenate([[0], np.cumsum(nrec)[:-1]])
    # last record of every block ends at 16 * nrec of that block
    assert np.array_equal(ke[rb + nrec - 1], 16 * nrec.astype(np.uint32))


def test_workspace_reuse_across_batch_sizes(oracle):
    """One workspace (zero-filled once) serves a sequence of batches of different sizes and
    both entry points: the launch-parity look-back slots are cleared by the kernels
    themselves (no per-call fill), so stale words from a bigger earlier batch must never
    leak into a later one."""
    codec = _dev()
    import torch
    from mtblx import synth
    data, off, ln = synth.cfg2_file(6000)
    ws = codec.Workspace(6000)
    exp_all = oracle.decode_blocks(data, off, ln)
    for n in (6000, 37, 6000, 1, 2500, 6000, 13, 6000):
        o, l_ = off[:n], ln[:n]
        batch = codec.DeviceBatch.from_host(data, o, l_)
        probe = codec.DecodedBlocks(batch.nblk, 0, 0, 0)
        codec.count_blocks(batch, probe, ws)
        torch.cuda.synchronize()
        nr, kb, vb, fl = probe.totals_host()
        assert fl == 0
        exp_nr = int(exp_all.nrec[:n].sum())
        assert nr == exp_nr, (n, nr, exp_nr)
        out = codec.DecodedBlocks(batch.nblk, nr, kb, vb)
        codec.decode_into(batch, out, ws)
        torch.cuda.synchronize()
        dev = out.to_host()
        orc = oracle.decode_blocks(data, o, l_)
        assert_same(dev, orc, n)


def test_64k_blocks_cfg2_scheme(oracle):
    """cfg4's 64 KiB leg (cfg2 key/value scheme): k_decode_pipe<PipeLarge>."""
    from mtblx import synth
    data, off, ln = synth.cfg2_file(300, block_size=65536)
    assert int(ln.max()) > 60000
    orc = oracle.decode_blocks(data, off, ln)
    dev = device_decode(data, off, ln)
    assert_same(dev, orc, off.size)
    assert (orc.status == 0).all()


def test_64k_blocks_long_keys(oracle):
    """cfg3-like 64 KiB blocks: 8..256 B keys (multi-byte varint headers for long suffixes),
    64 B values, and a few mutated copies."""
    rng = np.random.default_rng(21)
    blocks = []
    for _ in range(24):
        n = int(rng.integers(150, 330))
        recs = corpus.random_records(rng, n, 8, 256, 64, 64)
        b = oracle.build_block(recs)
        if len(b) <= 65000:
            blocks.append(b)
    assert len(blocks) >= 8 and max(len(b) for b in blocks) > 40000
    big = list(blocks)
    mut = [corpus.mutate(rng, b) for b in blocks[:8]]
    orc = run_both(oracle, big + mut, rng=np.random.default_rng(3))
    assert (orc.status[: len(big)] == 0).all()


def test_crc32c_blocks_vs_oracle(oracle):
    """f1: device CRC-32C of block contents == crate crc32c (oracle), and the framed check
    flags exactly the blocks whose stored checksum was corrupted."""
    codec = _dev()
    import torch
    from mtblx import synth
    data, off, ln = synth.cfg2_file(3000)
    rng = np.random.default_rng(8)
    # varied block sizes including < 64 B and 64 KiB contents (unframed)
    extra = [bytes(rng.integers(0, 256, int(n), dtype=np.uint8)) for n in (0, 1, 3, 4, 5, 63, 64, 65, 1000, 65000, 300000)]
    xd, xo, xl = corpus.pack(extra, rng=rng, lead=3)
    for d_, o_, l_, framed in ((data, off, ln, True), (xd, xo, xl, False)):
        batch = codec.DeviceBatch.from_host(d_, o_, l_)
        crc, bad = codec.crc32c_blocks(batch, framed=framed)
        torch.cuda.synchronize()
        got = crc.cpu().numpy().view(np.uint32)
        exp = np.array([oracle.crc32c(bytes(d_[int(o): int(o) + int(n)])) for o, n in zip(o_, l_)], np.uint32)
        assert np.array_equal(got, exp)
        if framed:
            assert int(bad.sum().item()) == 0
    # corrupt the stored checksum of some blocks and one content byte of another
    d2 = data.copy()
    for b in (5, 77, 2999):
        d2[int(off[b]) - 2] ^= 0x40
    d2[int(off[1234]) + 100] ^= 1
    batch = codec.DeviceBatch.from_host(d2, off, ln)
    _, bad = codec.crc32c_blocks(batch, framed=True)
    torch.cuda.synchronize()
    assert sorted(np.nonzero(bad.cpu().numpy())[0].tolist()) == [5, 77, 1234, 2999]


def test_fused_verify_decode(oracle):
    """f1 fused: decode + CRC-32C in one launch == the plain decode (all outputs) and the
    oracle's crc32c of every block; the framed check flags exactly the corrupted checksums.
    Shapes: cfg2 (PipeSmall), builder / quirk / mutated blocks incl. < 4 B and < 64 B blocks,
    blocks too large for a staging slot (HBM path), 64 KiB blocks (PipeLarge), > 64 KiB
    blocks (separate-launch fallback)."""
    codec = _dev()
    import torch
    from mtblx import synth
    rng = np.random.default_rng(77)
    cases = []
    data, off, ln = synth.cfg2_file(3000)
    d2 = data.copy()
    for b in (0, 7, 1500, 2999):
        d2[int(off[b]) - 1] ^= 0x08
    cases.append((d2, off, ln, True, [0, 7, 1500, 2999]))
    blocks = corpus.builder_blocks(oracle, seed=71, count=120, max_bytes=9000) + \
        [b for _, b, _ in corpus.quirk_blocks()] + corpus.mutated_blocks(oracle, seed=72, count=150)
    blocks += [bytes(rng.integers(0, 256, int(n), dtype=np.uint8)) for n in (0, 1, 2, 3, 4, 5, 63, 64, 65, 127, 128)]
    for n in (400, 700):   # > the PipeSmall slot of this batch's mix: unstaged, CRC from HBM
        blocks.append(oracle.build_block(corpus.random_records(rng, n, 4, 60, 10, 120)))
    d, o, l = corpus.pack(blocks, rng=rng, lead=3)
    cases.append((d, o, l, False, []))
    d, o, l = synth.cfg2_file(200, block_size=65536)
    cases.append((d, o, l, True, []))
    for bs in (16384, 32768):   # PipeSmall tiles of fewer blocks than copy waves: window rounds split
        d, o, l = synth.cfg2_file(150, block_size=bs)
        d = d.copy()
        d[int(o[3]) - 2] ^= 0x40
        cases.append((d, o, l, True, [3]))
    big = [oracle.build_block(corpus.random_records(rng, 1400, 8, 60, 40, 60)) for _ in range(3)]
    assert max(len(b) for b in big) > 70000
    d, o, l = corpus.pack(big, rng=rng)
    cases.append((d, o, l, False, []))
    for (d_, o_, l_, framed, bad_exp), fused in [(c, f) for c in cases for f in (True, False)]:
        batch = codec.DeviceBatch.from_host(d_, o_, l_)
        out, crc, bad = codec.decode_verify(batch, framed=framed, fused=fused)
        torch.cuda.synchronize()
        dev = out.to_host()
        orc = oracle.decode_blocks(d_, o_, l_)
        assert_same(dev, orc, o_.size) if (orc.status != 5).all() else None
        got = crc.cpu().numpy().view(np.uint32)
        exp = np.array([oracle.crc32c(bytes(d_[int(a): int(a) + int(n)])) for a, n in zip(o_, l_)], np.uint32)
        assert np.array_equal(got, exp), np.nonzero(got != exp)[0][:10]
        assert sorted(np.nonzero(bad.cpu().numpy())[0].tolist()) == (bad_exp if framed else [])



def _block_of_len(oracle, rng, L, iv, n, kmax):
    """a BlockBuilder block of exactly L bytes: n records, keys 4..kmax B, the value bytes spread
    so the content reaches L (the last value absorbs the varint-length steps)"""
    recs = corpus.random_records(rng, n, 4, kmax, 0, 0)
    need = L - len(oracle.build_block(recs, restart_interval=iv))
    assert need >= 0
    vl = [need // n] * n
    for _ in range(8):
        vl[-1] = max(0, vl[-1])
        cur = [(k, bytes(rng.integers(0, 256, v, dtype=np.uint8))) for (k, _), v in zip(recs, vl)]
        b = oracle.build_block(cur, restart_interval=iv)
        if len(b) == L:
            return b
        vl[-1] += L - len(b)
    raise AssertionError("block length not reached")


def test_pipelarge_max_shapes(oracle):
    """PipeLarge / PipeLargeV at their largest tile and block shapes, fused verify and
    decode + CRC against the oracle: blocks of exactly the largest PipeLarge slot (65 601 B: one
    per 65 664 B tile) with 64 restart intervals (the tile's interval capacity), 65 (one past),
    one restart per entry, and a few long values; then blocks of 32 785 B (the largest two per
    tile) with 32 intervals each (64 per tile)."""
    codec = _dev()
    import torch
    rng = np.random.default_rng(2026)
    batches = [
        [_block_of_len(oracle, rng, 65601, 16, 1024, 24), _block_of_len(oracle, rng, 65601, 16, 1025, 24),
         _block_of_len(oracle, rng, 65601, 1, 200, 40), _block_of_len(oracle, rng, 65601, 16, 40, 60),
         _block_of_len(oracle, rng, 65601, 16, 300, 300), _block_of_len(oracle, rng, 60000, 7, 900, 30)],
        [_block_of_len(oracle, rng, 32785, 16, 512, 24) for _ in range(5)] + [_block_of_len(oracle, rng, 32785, 1, 100, 40)],
    ]
    for blocks in batches:
        blocks = blocks * 3
        d, o, l = corpus.pack(blocks, rng=rng, lead=5)
        for fused in (True, False):
            batch = codec.DeviceBatch.from_host(d, o, l)
            out, crc, bad = codec.decode_verify(batch, framed=False, fused=fused)
            torch.cuda.synchronize()
            dev = out.to_host()
            orc = oracle.decode_blocks(d, o, l)
            assert (orc.status == 0).all()
            assert_same(dev, orc, o.size)
            exp = np.array([oracle.crc32c(b) for b in blocks], np.uint32)
            assert np.array_equal(crc.cpu().numpy().view(np.uint32), exp)
            assert not bad.cpu().numpy().any()


def _tail_records(rng, n, mode):
    """n strictly increasing keys for the copy waves' key-tail paths, random 0..64 B values.
    "counter": be64 counter with random gaps (shared ~5 B) + a random tail of 0..292 B, so every
    key byte past 16 is the entry's own suffix (the dense chunk list); "p16": a common 16-byte
    prefix, one distinct byte, a tail (shared == 16 exactly: the dense path's boundary; n <= 256);
    "mixed": counter keys, every third one repeating the previous key's first 20..60 bytes
    (shared > 16 in some rows of a wave: the per-plane path)."""
    lens = [0, 1, 8, 9, 16, 17, 24, 31, 32, 33, 48, 100, 160, 240, 292]
    keys, c, prev = [], 0, b""
    p16 = bytes(rng.integers(0, 256, 16, dtype=np.uint8))
    for i in range(n):
        tail = bytes(rng.integers(0, 256, int(rng.choice(lens)), dtype=np.uint8))
        if mode == "p16":
            k = p16 + bytes([i]) + tail
        elif mode == "mixed" and len(prev) > 24 and rng.random() < 0.35:
            cut = int(rng.integers(20, min(60, len(prev)) + 1))
            k = prev[:cut] + b"\xff" + tail   # > prev: byte `cut` of prev is < 0xff or prev ends there
            if k <= prev:
                k = prev + b"\x01"
        else:
            c += int(rng.integers(1, 1 << 20))
            k = c.to_bytes(8, "big") + tail
            if k <= prev:
                k = prev + b"\x02"
        keys.append(k)
        prev = k
    assert all(a < b for a, b in zip(keys, keys[1:]))
    return [(k, bytes(rng.integers(0, 256, int(rng.integers(0, 65)), dtype=np.uint8))) for k in keys]


def test_key_tails_dense_and_planes(oracle):
    """Keys longer than 16 B through both copy paths: the wave-wide dense chunk list (no live
    entry of the wave inherits a byte past 16) and the per-plane scan (some entry does), in
    ~4 KiB blocks (PipeSmall) and ~40-64 KiB blocks (PipeLarge), restart intervals 16, 1, 7, 13."""
    rng = np.random.default_rng(0x7a11)
    for nrec in (36, 560):
        blocks = []
        for mode in ("counter", "p16", "mixed"):
            for iv in (16, 16, 1, 7, 13):
                recs = _tail_records(rng, min(nrec, 256) if mode == "p16" else nrec, mode)
                blocks.append(oracle.build_block(recs, restart_interval=iv))
        blocks = [b for b in blocks if len(b) <= 65000] * 4
        assert nrec < 100 or max(len(b) for b in blocks) > 49200   # PipeLarge
        orc = run_both(oracle, blocks, rng=np.random.default_rng(5))
        assert (orc.status == 0).all()
        assert int(np.diff(orc.key_end.astype(np.int64)).max()) > 200


def test_pipelarge_walk_modes_alternate(oracle):
    """PipeLarge's walker picks its first interval walk from the previous tile (1-byte headers ->
    walk_pos, 2-byte -> walk_pos2).  One batch alternates 64 KiB-class blocks of 16 B keys
    (1-byte headers), long-key blocks (2-byte non_shared varints), blocks with 20 KB values
    (3-byte varints: the careful walk) and corrupted copies, so the mode flips both ways."""
    from mtblx import synth
    rng = np.random.default_rng(0x3a1c)
    d2, o2, l2 = synth.cfg2_file(12, block_size=65536)
    short = [bytes(d2[int(o): int(o) + int(n)]) for o, n in zip(o2, l2)]
    longk = []
    while len(longk) < 8:
        b = oracle.build_block(_tail_records(rng, 520, "counter"), restart_interval=16)
        if 49200 < len(b) <= 65000:
            longk.append(b)
    big = []
    for _ in range(3):
        recs = corpus.random_records(rng, 40, 8, 24, 16, 64)
        k, _ = recs[17]
        recs[17] = (k, bytes(rng.integers(0, 256, 20000, dtype=np.uint8)))
        big.append(oracle.build_block(recs, restart_interval=16))
    blocks = []
    for i in range(12):
        blocks.append(short[i])
        if i < 8:
            blocks.append(longk[i])
        if i % 4 == 1:
            blocks.append(big[i // 4])
        if i % 3 == 2:
            blocks.append(corpus.mutate(rng, longk[i % 8]))
    assert max(len(b) for b in blocks) > 49200 and max(len(b) for b in blocks) <= 65600
    orc = run_both(oracle, blocks, rng=np.random.default_rng(9))
    assert int((orc.status == 0).sum()) >= 23


def test_pipelarge_tile_counts_one_workspace(oracle):
    """PipeLarge's late-walk pipeline with 1, 2, 3, 257 and 513 tiles (workgroups with 1..3 tiles:
    the fill and drain of the two-buffer schedule), one workspace reused across the batches, and
    long-key blocks mixed in so the walk order switches mid-launch."""
    codec = _dev()
    import torch
    from mtblx import synth
    data, off, ln = synth.cfg2_file(513, block_size=65536)
    rng = np.random.default_rng(0x1a7e)
    longk = []
    while len(longk) < 4:
        b = oracle.build_block(_tail_records(rng, 520, "counter"), restart_interval=16)
        if 49200 < len(b) <= 65000:
            longk.append(b)
    blocks = [bytes(data[int(o): int(o) + int(n)]) for o, n in zip(off, ln)]
    for i, b in enumerate(longk):
        blocks[100 * i + 7] = b
    d, o, l = corpus.pack(blocks)
    ws = codec.Workspace(len(blocks))
    exp_all = oracle.decode_blocks(d, o, l)
    assert (exp_all.status == 0).all()
    for n in (1, 2, 3, 257, 513, 2):
        batch = codec.DeviceBatch.from_host(d, o[:n], l[:n])
        probe = codec.DecodedBlocks(batch.nblk, 0, 0, 0)
        codec.count_blocks(batch, probe, ws)
        torch.cuda.synchronize()
        nr, kb, vb, fl = probe.totals_host()
        assert fl == 0 and nr == int(exp_all.nrec[:n].sum())
        out = codec.DecodedBlocks(batch.nblk, nr, kb, vb)
        codec.decode_into(batch, out, ws)
        torch.cuda.synchronize()
        assert_same(out.to_host(), oracle.decode_blocks(d, o[:n], l[:n]), n)


@pytest.mark.parametrize("block_size", [4096, 65536])
def test_directory_in_any_order(oracle, block_size):
    """The directory is the caller's: windows out of file order, repeated, overlapping, or
    pointing into another block (a corrupt index does all of these, src/reader.rs:177-186).
    A tile whose blocks do not all lie in [first start, last end) must not be staged as one
    contiguous range (it was: a block before its tile's first one was read at a wrapped stage
    offset).  PipeSmall (4 KiB) and PipeLarge (64 KiB) batches, plain and fused-verify."""
    codec = _dev()
    import torch
    from mtblx import synth
    rng = np.random.default_rng(block_size)
    data, off, ln = synth.cfg2_file(400 if block_size == 4096 else 60, block_size=block_size)
    n = off.size
    o2, l2 = off.astype(np.uint64).copy(), ln.astype(np.uint32).copy()
    perm = rng.permutation(n)
    o2, l2 = o2[perm], l2[perm]                              # out of file order
    for _ in range(n // 8):                                  # windows inside other blocks
        i, j = int(rng.integers(0, n)), int(rng.integers(0, n))
        sh = int(rng.integers(1, max(2, int(l2[j]) // 2)))
        o2[i] = o2[j] + sh
        l2[i] = int(rng.integers(0, max(1, int(l2[j]) - sh)))
    o2 = np.concatenate([o2, o2[:5], np.sort(o2)[:7]])       # repeated entries
    l2 = np.concatenate([l2, l2[:5], l2[np.argsort(o2[:n])][:7]])
    orc = oracle.decode_blocks(data, o2, l2)
    assert_same(device_decode(data, o2, l2), orc, o2.size)
    batch = codec.DeviceBatch.from_host(data, o2, l2)
    out, crc, bad = codec.decode_verify(batch, framed=False, fused=True)
    torch.cuda.synchronize()
    assert_same(out.to_host(), orc, o2.size)
    exp = np.array([oracle.crc32c(bytes(data[int(a): int(a) + int(b)])) for a, b in zip(o2, l2)], np.uint32)
    assert np.array_equal(crc.cpu().numpy().view(np.uint32), exp)
