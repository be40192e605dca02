"""Robustness of the device decode: launches that must never hand back wrong records.

- A tile whose aggregate does not fit the packed look-back word (>= 2^21 value bytes or records in
  one tile: one block > 64 KiB is one tile of k_decode_tiles) publishes exact side words; every
  later tile's bases must still equal the oracle's.
- A look-back timeout (include/mtblx.h, totals[3] bit 1) is rejected by every reader surface:
  codec (Python), Reader (Python), HostPipe (C ABI, synchronous: re-runs the chunk once, then
  MTBLX_E_TIMEOUT) and the C++ surface (include/mtbl.hpp, through the `dump` example).  The
  timeout is injected with the library's MTBLX_DEBUG_FLAGS test knob.
- A block window past the end of the data buffer: the reference's slice panics (CORRUPT), the
  device reads nothing outside the buffer, and the framed checksum check reports it bad.
"""
import os
import subprocess

import numpy as np
import pytest

import corpus

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _codec():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from mtblx import codec
    return codec


def _decode(data, off, ln):
    codec = _codec()
    import torch
    out = codec.decode_blocks(codec.DeviceBatch.from_host(data, off, ln))
    torch.cuda.synchronize()
    return out.to_host()


def _assert_same(dev, orc):
    for k in ("status", "nrec", "rec_base", "key_base", "val_base", "key_end", "val_end", "keys", "vals"):
        a, b = getattr(dev, k), getattr(orc, k)
        assert np.array_equal(a, b), (k, np.nonzero(a != b)[0][:8] if a.shape == b.shape else (a.shape, b.shape))
    assert dev.totals[3] == 0


def test_tile_aggregate_exact_words(oracle):
    """an early block holding a >= 2 MiB value, and one holding >= 2^21
    records, ahead of ordinary blocks in the same batch."""
    rng = np.random.default_rng(41)
    big_val = oracle.build_block([(b"k0", rng.integers(0, 256, (5 << 19) + 77, dtype=np.uint8).tobytes()),
                                  (b"k1", b"v")])
    n = (1 << 21) + 4321
    many = oracle.build_block([(i.to_bytes(3, "big"), b"") for i in range(n)])
    rest = corpus.builder_blocks(oracle, seed=42, count=30, max_bytes=9000)
    blocks = [big_val, rest[0], many] + rest[1:]
    data, off, ln = corpus.pack(blocks, rng=rng)
    orc = oracle.decode_blocks(data, off, ln)
    assert int(orc.nrec[2]) == n and int(orc.val_base[1] - orc.val_base[0]) >= (1 << 21)
    _assert_same(_decode(data, off, ln), orc)


def test_window_past_buffer_is_corrupt(oracle):
    """blk_off + blk_len > data_len -> MTBLX_ST_CORRUPT with no records (the
    reference's BytesView::slice panics), for the pipelined (4 KiB) and the exact (> 64 KiB)
    kernels; in-bounds blocks are unaffected; the framed checksum check flags the block."""
    codec = _codec()
    import torch
    from mtblx import synth
    data, off, ln = synth.cfg2_file(200)
    rng = np.random.default_rng(43)
    big = [oracle.build_block(corpus.random_records(rng, 1500, 8, 60, 40, 60)) for _ in range(3)]
    bd, bo, bl = corpus.pack(big, rng=rng)
    for d_, o_, l_ in ((data, off, ln), (bd, bo, bl)):
        cut = int(o_[-1]) + int(l_[-1]) // 2     # the last block overhangs the buffer
        o2 = np.concatenate([o_, [cut + 100]]).astype(np.uint64)   # and one starts past it
        l2 = np.concatenate([l_, [64]]).astype(np.uint32)
        dd = d_[:cut].copy()
        dev = _decode(dd, o2, l2)
        nb = o_.size
        assert dev.status[nb - 1] == 2 and dev.status[nb] == 2 and dev.nrec[nb - 1] == 0 and dev.nrec[nb] == 0
        orc = oracle.decode_blocks(dd, o_[: nb - 1], l_[: nb - 1])
        assert np.array_equal(dev.status[: nb - 1], orc.status) and np.array_equal(dev.nrec[: nb - 1], orc.nrec)
        assert np.array_equal(dev.keys, orc.keys) and np.array_equal(dev.vals, orc.vals)
        assert np.array_equal(dev.key_end, orc.key_end) and np.array_equal(dev.val_end, orc.val_end)
        batch = codec.DeviceBatch.from_host(dd, o2, l2)
        _, bad = codec.crc32c_blocks(batch, framed=True)
        out, _, vbad = codec.decode_verify(batch, framed=True, fused=True)
        torch.cuda.synchronize()
        assert bad.cpu().numpy()[nb - 1:].tolist() == [1, 1]
        assert vbad.cpu().numpy()[nb - 1:].tolist() == [1, 1]


def test_fused_verify_window_far_past_buffer(oracle):
    """r05: the fused verify kernels read a block's stored checksum (the u32 before its content)
    from HBM.  For a window starting far past the buffer -- a corrupt index read with
    verification off points a block anywhere -- that read went to data + off - 4 unguarded (an
    access tens of MiB or a TiB past the allocation).  Every verify path must flag such blocks
    bad, decode them CORRUPT and read nothing outside the buffer; in-buffer blocks of the same
    tiles stay exact.  PipeSmallV (4 KiB blocks) and PipeLargeV (64 KiB blocks)."""
    codec = _codec()
    import torch
    from mtblx import synth
    for bs, nblk in ((4096, 300), (65536, 60)):
        data, off, ln = synth.cfg2_file(nblk, block_size=bs)
        n = off.size
        far = [len(data) + (8 << 20), 1 << 40, (1 << 40) + 4]
        o2 = off.astype(np.uint64).copy()
        l2 = ln.astype(np.uint32).copy()
        idx = [5, n // 2, n - 1]
        for i, f in zip(idx, far):
            o2[i] = f
        batch = codec.DeviceBatch.from_host(data, o2, l2)
        for fused in (True, False):
            out, crc, bad = codec.decode_verify(batch, framed=True, fused=fused)
            torch.cuda.synchronize()
            dev = out.to_host()
            b = bad.cpu().numpy()
            assert sorted(np.nonzero(b)[0].tolist()) == idx, (bs, fused)
            assert all(dev.status[i] == 2 and dev.nrec[i] == 0 for i in idx)
            keep = [i for i in range(n) if i not in idx]
            orc = oracle.decode_blocks(data, off[keep], ln[keep])
            assert np.array_equal(dev.status[keep], orc.status) and np.array_equal(dev.nrec[keep], orc.nrec)
            assert np.array_equal(dev.keys, orc.keys) and np.array_equal(dev.vals, orc.vals)
            got = crc.cpu().numpy().view(np.uint32)[keep]
            exp = np.array([oracle.crc32c(bytes(data[int(off[i]): int(off[i]) + int(ln[i])])) for i in keep], np.uint32)
            assert np.array_equal(got, exp)


def test_lookback_timeout_rejected_everywhere(oracle, monkeypatch, tmp_path):
    """no API hands back records from a launch whose look-back timed out."""
    codec = _codec()
    import torch
    from mtblx import pipe, reader, synth
    from mtblx.writer import Writer
    data, off, ln = synth.cfg2_file(300)
    w = Writer(4096, 16)
    for k, v in synth.cfg1_records(2000):
        w.insert(k, v)
    fbytes = w.into_inner()
    path = tmp_path / "f.mtbl"
    path.write_bytes(fbytes)
    batch = codec.DeviceBatch.from_host(data, off, ln)
    # sanity: without the knob everything decodes
    out = codec.decode_blocks(batch)
    torch.cuda.synchronize()
    nr, kb, vb, fl = out.totals_host()
    assert fl == 0
    monkeypatch.setenv("MTBLX_DEBUG_FLAGS", "2")
    # codec: the count pass and the decode both report it
    with pytest.raises(codec.LaunchTimeout):
        codec.decode_blocks(batch)
    ws = codec.Workspace(batch.nblk)
    codec.decode_into(batch, out, ws)
    torch.cuda.synchronize()
    with pytest.raises(codec.LaunchTimeout):
        out.to_host()
    assert out.totals_host(check=False)[3] & 2
    # Reader (index decode at open)
    with pytest.raises(codec.LaunchTimeout):
        reader.Reader(fbytes).iter()
    # end-to-end pipe: the chunk is re-run once, then MTBLX_E_TIMEOUT
    ho = pipe.HostOutputs(off.size, nr, kb, vb)
    with pytest.raises(codec.LaunchTimeout):
        pipe.HostPipe().decode(data, off, ln, ho)
    # C++ surface
    dump = os.path.join(ROOT, "oxidized-mtbl_amd", "build", "dump")
    if os.path.exists(dump):
        r = subprocess.run([dump, str(path)], capture_output=True, timeout=120, env=dict(os.environ))
        assert r.returncode == 1 and b"look-back timeout" in r.stderr, r
        assert r.stdout == b""
    monkeypatch.delenv("MTBLX_DEBUG_FLAGS")
    # and the same workspace works again afterwards
    codec.decode_into(batch, out, ws)
    torch.cuda.synchronize()
    assert out.totals_host() == (nr, kb, vb, 0)
    if os.path.exists(dump):
        r = subprocess.run([dump, str(path)], capture_output=True, timeout=120)
        assert r.returncode == 0 and r.stdout.count(b"\n") == 2000


def test_timeout_before_tile0_survives(oracle, monkeypatch):
    """tile 0's walker zeroes totals[3] right before it publishes A(0); a
    workgroup whose look-back on A(0) gave up BEFORE that (workgroup 0 late / not resident) must
    still see its timeout reported.  Knobs: the bounded waits give up after 20 ms and tile 0's
    walker publishes 300 ms late, so every other workgroup's first look-back times out first."""
    codec = _codec()
    import torch
    from mtblx import synth
    data, off, ln = synth.cfg2_file(600)          # 50 tiles: one round of look-backs on A(0)
    batch = codec.DeviceBatch.from_host(data, off, ln)
    ref = codec.decode_blocks(batch)
    torch.cuda.synchronize()
    tot = ref.totals_host()
    assert tot[3] == 0
    ws = codec.Workspace(batch.nblk)
    out = codec.decode_blocks(batch)              # outputs of the right size
    torch.cuda.synchronize()
    monkeypatch.setenv("MTBLX_DEBUG_WAIT_MS", "20")
    monkeypatch.setenv("MTBLX_DEBUG_DELAY0_MS", "300")
    codec.decode_into(batch, out, ws)
    torch.cuda.synchronize()
    assert out.totals_host(check=False)[3] & 2
    with pytest.raises(codec.LaunchTimeout):
        out.to_host()
    monkeypatch.delenv("MTBLX_DEBUG_DELAY0_MS")
    monkeypatch.delenv("MTBLX_DEBUG_WAIT_MS")
    codec.decode_into(batch, out, ws)             # the workspace and outputs work again
    torch.cuda.synchronize()
    assert out.totals_host() == tot
    h, r = out.to_host(), ref.to_host()
    assert np.array_equal(h.keys, r.keys) and np.array_equal(h.key_end, r.key_end)


@pytest.mark.gpu
def test_workspace_one_launch_at_a_time(monkeypatch):
    """the workspace's launch-parity protocol (decode.hip ws_begin: parity from
    the epoch the previous launch left; the other parity's slots cleared for the next launch) holds
    only in stream order.  The surface enforces it: a launch on stream B while stream A's launch on
    the same workspace is still running is refused (WorkspaceBusy, nothing launched), not run into
    the other launch's look-back words.  Stream A's launch is held ~300 ms by the debug knob that
    starts workgroup 0 late (the look-back waits on it; no timeout at the default bound)."""
    if os.environ.get("MTBLX_BOUNDS_CHECK"):
        pytest.skip("the bounds-checked build synchronizes every launch: two launches never overlap")
    codec = _codec()
    import torch
    from mtblx import synth
    data, off, ln = synth.cfg2_file(600)
    batch = codec.DeviceBatch.from_host(data, off, ln)
    ref = codec.decode_blocks(batch)
    torch.cuda.synchronize()
    ws = codec.Workspace(batch.nblk)
    out_a, out_b = codec.decode_blocks(batch), codec.decode_blocks(batch)
    torch.cuda.synchronize()
    sa, sb = torch.cuda.Stream(), torch.cuda.Stream()
    monkeypatch.setenv("MTBLX_DEBUG_DELAY0_MS", "300")
    codec.decode_into(batch, out_a, ws, sa)
    monkeypatch.delenv("MTBLX_DEBUG_DELAY0_MS")
    with pytest.raises(codec.WorkspaceBusy):
        codec.decode_into(batch, out_b, ws, sb)
    with pytest.raises(codec.WorkspaceBusy):
        codec.count_blocks(batch, out_b, ws, sb)
    codec.decode_into(batch, out_a, ws, sa)       # the same stream: ordered after it, allowed
    sa.synchronize()
    codec.decode_into(batch, out_b, ws, sb)       # A is done: B may take the workspace
    torch.cuda.synchronize()
    for o in (out_a, out_b):
        assert o.totals_host() == ref.totals_host()
        h, r = o.to_host(), ref.to_host()
        assert np.array_equal(h.keys, r.keys) and np.array_equal(h.vals, r.vals) and np.array_equal(h.key_end, r.key_end)


@pytest.mark.gpu
def test_poison_fill_is_active():
    """MTBLX_POISON=1 runs (tests/conftest.py): fresh device allocations really are all-ones"""
    if not os.environ.get("MTBLX_POISON"):
        pytest.skip("poison mode off")
    _codec()
    import torch
    assert bool((torch.empty(4096, dtype=torch.uint8, device="cuda") == 255).all().item())
    assert bool((torch.empty(64, dtype=torch.int64, device="cuda") == (1 << 63) - 1).all().item())
    assert os.environ.get("MTBLX_DEBUG_POISON") == "1"
