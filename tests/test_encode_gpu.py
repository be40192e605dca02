"""Device encode (Writer block cut + BlockBuilder + write_block framing) vs the oracle and
the product host Writer (itself byte-identical to the oracle Writer, which the golden files pin).

- framed blocks == the data-block region of the file the Writer writes, byte for byte
- unframed block contents == oracle_build_block (src/block_builder.rs restated) per block
- decode(encode(x)) == x on the cfg3 scheme (Zipf 8..256 B keys, 64 KiB blocks)
- Writer panics (out-of-order key, interval 0) are reported, never produced
"""
import numpy as np
import pytest

import corpus

pytestmark = pytest.mark.gpu


def _enc():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from mtblx import encode
    return encode


def _writer_file(recs, block_size, interval):
    from mtblx.writer import Writer
    w = Writer(block_size, interval)
    for k, v in recs:
        w.insert(k, v)
    data = w.into_inner()
    off, ln = w.block_dir
    return data, off, ln, w.block_nrec


def test_framed_equals_writer_file(oracle):
    enc = _enc()
    rng = np.random.default_rng(61)
    cases = [(1024, 16, 300, 0, 30, 0, 40), (4096, 16, 3000, 0, 80, 0, 200), (8192, 3, 2000, 0, 300, 0, 50),
             (65536, 16, 6000, 8, 256, 64, 64), (2000, 1, 800, 0, 20, 0, 10), (4096, 40, 2500, 1, 60, 0, 120)]
    for bs, iv, n, kmin, kmax, vmin, vmax in cases:
        recs = corpus.random_records(rng, n, kmin, kmax, vmin, vmax)
        data, off, ln, nrec = _writer_file(recs, bs, iv)
        d = enc.DeviceRecords.from_list(recs)
        blk = enc.plan(d, bs, iv).cpu().numpy()
        assert blk.size - 1 == off.size, (bs, iv, blk.size - 1, off.size)
        assert np.array_equal(np.diff(blk), nrec.astype(np.int64))
        e = enc.encode_blocks(d, enc.plan(d, bs, iv), iv, framed=True)
        total = int(e.totals[0].item())
        assert int(e.totals[1].item()) == 0 and (e.status.cpu().numpy() == 0).all()
        idx_off = int(np.frombuffer(data[-512:-504], np.uint64)[0])
        assert total == idx_off
        assert e.out[:total].cpu().numpy().tobytes() == data[:idx_off]
        assert np.array_equal(e.blk_off.cpu().numpy().astype(np.uint64), off)
        assert np.array_equal(e.blk_len.cpu().numpy().astype(np.uint32), ln)
        # the oracle reads the device-written blocks back (its own CRC + decode)
        orc = oracle.decode_blocks(e.out[:total].cpu().numpy(), off, ln)
        assert (orc.status == 0).all() and int(orc.nrec.sum()) == n


def test_unframed_blocks_equal_oracle_builder(oracle):
    enc = _enc()
    import torch
    rng = np.random.default_rng(62)
    for iv in (1, 2, 5, 16, 17, 40):
        recs = corpus.random_records(rng, 1500, 0, 120, 0, 90)
        d = enc.DeviceRecords.from_list(recs)
        # arbitrary block cuts (not the Writer's): 0-record blocks included
        cuts = np.sort(rng.integers(0, len(recs) + 1, 40))
        blk = torch.tensor(np.concatenate([[0], cuts, [len(recs)]]), dtype=torch.int64, device="cuda")
        e = enc.encode_blocks(d, blk, iv, framed=False)
        out = e.out.cpu().numpy()
        bo, bl = e.blk_off.cpu().numpy(), e.blk_len.cpu().numpy()
        b = blk.cpu().numpy()
        for j in range(b.size - 1):
            exp = oracle.build_block(recs[b[j]: b[j + 1]], restart_interval=iv)
            assert out[bo[j]: bo[j] + bl[j]].tobytes() == exp, (iv, j)
    # interval 0: one-record blocks encode ([0, 0] restarts), two-record blocks panic
    recs = corpus.random_records(rng, 10, 1, 10, 0, 10)
    d = enc.DeviceRecords.from_list(recs)
    blk = torch.tensor([0, 1, 2, 4, 5], dtype=torch.int64, device="cuda")
    e = enc.encode_blocks(d, blk, 0, framed=False)
    st = e.status.cpu().numpy()
    assert st.tolist() == [0, 0, 2, 0]
    out = e.out.cpu().numpy()
    for j in (0, 1, 3):
        o, n_ = int(e.blk_off[j].item()), int(e.blk_len[j].item())
        assert out[o: o + n_].tobytes() == oracle.build_block(recs[int(blk[j]): int(blk[j + 1])], restart_interval=0)


def test_writer_panics_reported():
    enc = _enc()
    import torch
    recs = [(b"b", b"1"), (b"a", b"2")]
    with pytest.raises(enc.WriterPanic) as ei:
        enc.plan(enc.DeviceRecords.from_list(recs), 4096, 16)
    assert ei.value.flags & 1
    recs = [(bytes([i]), b"x") for i in range(1, 50)]
    with pytest.raises(enc.WriterPanic) as ei:
        enc.plan(enc.DeviceRecords.from_list(recs), 4096, 0)
    assert ei.value.flags & 2
    # equal keys are out of order too (key <= last_key)
    with pytest.raises(enc.WriterPanic):
        enc.plan(enc.DeviceRecords.from_list([(b"a", b""), (b"a", b"")]), 4096, 16)
    del torch


def test_shards_are_independent_writers():
    enc = _enc()
    import torch
    rng = np.random.default_rng(63)
    recs = corpus.random_records(rng, 4000, 0, 50, 0, 100)
    cuts = [0, 700, 701, 2500, 2500, 4000]
    d = enc.DeviceRecords.from_list(recs)
    blk = enc.plan(d, 2048, 8, shard_rec=torch.tensor(cuts, dtype=torch.int64, device="cuda")).cpu().numpy()
    exp = []
    for a, b in zip(cuts[:-1], cuts[1:]):
        if b > a:
            _, _, _, nrec = _writer_file(recs[a:b], 2048, 8)
            exp.append(a + np.concatenate([[0], np.cumsum(nrec)[:-1]]))
    assert np.array_equal(blk[:-1], np.concatenate(exp)) and blk[-1] == 4000


def _plan_serial(recs, shard_rec, bs, iv, cap):
    """the round-1..4 block cut (one wave per shard walking the Writer's chain), exported as
    mtblx_encode_plan_serial: the parallel planner must cut exactly where it does"""
    import ctypes as C
    import torch
    from mtblx import _lib, codec
    L = _lib.lib()
    f = L.mtblx_encode_plan_serial
    f.argtypes = L.mtblx_encode_plan.argtypes
    f.restype = C.c_int
    blk = torch.empty(cap, dtype=torch.int64, device="cuda")
    nb, fl = C.c_uint64(0), C.c_uint32(0)
    rc_ = recs.cstruct()
    nsh = int(shard_rec.numel()) - 1
    ws = torch.empty(int(L.mtblx_plan_serial_workspace_bytes(nsh)), dtype=torch.uint8, device="cuda")
    rc = f(C.byref(rc_), C.c_void_p(shard_rec.data_ptr()), nsh, bs, iv, C.c_void_p(blk.data_ptr()),
           cap, C.byref(nb), C.byref(fl), C.c_void_p(ws.data_ptr()), ws.numel(), C.c_void_p(codec._stream_handle(None)))
    return rc, int(fl.value), blk[: int(nb.value) + 1].cpu().numpy()


def test_plan_caller_workspace_and_concurrent_cuts():
    """The block cut keeps no state of its own (include/mtblx.h: re-entrant, caller-owned
    workspace): two host threads on two streams cut two different cfg3 record
    sets at once, each with its own PlanWorkspace, and both equal the serial walk; a workspace too
    small for the parallel cut takes the serial walk (same cut); NULL, misaligned or (keep mode)
    too small are MTBLX_E_INVAL."""
    enc = _enc()
    import ctypes as C
    import threading
    import torch
    from mtblx import _lib, codec, synth
    L = _lib.lib()
    sets = [synth.cfg3_records_device(300_000, seed=41 + i)[0] for i in range(2)]
    cuts = [torch.tensor(c, dtype=torch.int64, device="cuda") for c in ([0, 100_000, 300_000], [0, 300_000])]
    exp = [_plan_serial(r, c, 65536, 16, 300_002) for r, c in zip(sets, cuts)]
    assert all(e[0] == 0 for e in exp)
    streams = [torch.cuda.Stream() for _ in sets]
    wss = [enc.PlanWorkspace(r.n, int(c.numel()) - 1, 16, keep) for r, c, keep in zip(sets, cuts, (True, False))]
    got, errs = [None, None], []
    torch.cuda.synchronize()

    def run(i):
        try:
            for _ in range(4):
                with torch.cuda.stream(streams[i]):
                    r = enc.plan(sets[i], 65536, 16, shard_rec=cuts[i], stream=streams[i], keep=(i == 0),
                                 workspace=wss[i])
                b = r[0] if i == 0 else r
                streams[i].synchronize()
                got[i] = b.cpu().numpy()
                assert np.array_equal(got[i], exp[i][2]), i
        except Exception as ex:   # noqa: BLE001 -- reported below
            errs.append(ex)

    th = [threading.Thread(target=run, args=(i,)) for i in range(2)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    assert not errs, errs
    # a workspace too small for the parallel cut: the serial walk, same cut
    small = enc.PlanWorkspace(sets[1].n, 1, 16, serial=True)
    assert np.array_equal(enc.plan(sets[1], 65536, 16, shard_rec=cuts[1], workspace=small).cpu().numpy(), exp[1][2])
    # keep mode has no serial fallback: a small workspace is MTBLX_E_INVAL
    with pytest.raises(RuntimeError, match="-1"):
        enc.plan(sets[1], 65536, 16, shard_rec=cuts[1], keep=True, workspace=small)
    # NULL and misaligned workspaces
    rc_ = sets[1].cstruct()
    blk = torch.empty(300_002, dtype=torch.int64, device="cuda")
    nb, fl = C.c_uint64(0), C.c_uint32(0)
    for ptr in (0, wss[1].ptr + 8):
        assert L.mtblx_encode_plan(C.byref(rc_), C.c_void_p(cuts[1].data_ptr()), 1, 65536, 16, C.c_void_p(blk.data_ptr()),
                                   300_002, C.byref(nb), C.byref(fl), C.c_void_p(ptr), wss[1].nbytes,
                                   C.c_void_p(codec._stream_handle(None))) == _lib.MTBLX_E_INVAL
    # the bound does not depend on the records: many tiny shards and one large one stay small
    b1 = int(L.mtblx_plan_workspace_bytes(1_000_000, 1, 16, 0))
    b2 = int(L.mtblx_plan_workspace_bytes(1_000_000, 50_000, 16, 0))
    assert b2 - b1 < 50_000 * 64


def test_parallel_plan_equals_writer_chain():
    """mtblx_encode_plan (r05: next(j) for every record from prefix sums + pointer doubling) cuts
    exactly where the Writer does (src/writer.rs:125-130, src/block_builder.rs:40-62): against
    the host Writer on small shapes, and against the serial device walk on large ones -- intervals
    1..5000, block sizes 1 KiB..1 MiB, values far larger than the block (a record alone past the
    size: one-record blocks), empty keys and values, empty and one-record shards, a shard of
    more than 4096 blocks (the next^4096 level), many shards."""
    enc = _enc()
    import torch
    from mtblx import synth
    rng = np.random.default_rng(64)
    for bs, iv, n, kmin, kmax, vmin, vmax in [(1024, 1, 500, 0, 30, 0, 40), (1024, 16, 600, 1, 20, 0, 3000),
                                              (4096, 7, 2000, 0, 80, 0, 200), (9000, 100, 3000, 0, 40, 0, 60),
                                              (1 << 20, 5000, 9000, 4, 60, 0, 300), (2048, 2, 1500, 0, 8, 0, 0),
                                              (1500, 16, 800, 1, 30, 900, 2500)]:
        recs = corpus.random_records(rng, n, kmin, kmax, vmin, vmax)
        _, _, _, nrec = _writer_file(recs, bs, iv)
        blk = enc.plan(enc.DeviceRecords.from_list(recs), bs, iv).cpu().numpy()
        assert np.array_equal(np.diff(blk), nrec.astype(np.int64)), (bs, iv)
    recs, _ = synth.cfg3_records_device(400_000, seed=9)
    dev = recs.key_end.device
    for bs, iv, cuts in [(65536, 16, [0, 400_000]), (1024, 16, [0, 400_000]), (4096, 3, [0, 1, 1, 2, 150_000, 150_000, 400_000]),
                         (30000, 40, list(np.linspace(0, 400_000, 101).astype(int))), (2048, 1, [0, 123_457, 400_000])]:
        sr = torch.tensor(cuts, dtype=torch.int64, device=dev)
        got = enc.plan(recs, bs, iv, shard_rec=sr).cpu().numpy()
        rc, fl, exp = _plan_serial(recs, sr, bs, iv, 400_002)
        assert rc == 0 and fl == 0
        assert np.array_equal(got, exp), (bs, iv, got.size, exp.size)
    # interval 0: only one-record blocks are legal; the parallel walk reports the panic too
    big = [(bytes([1, i]), bytes(3000)) for i in range(40)]
    blk = enc.plan(enc.DeviceRecords.from_list(big), 2048, 0).cpu().numpy()
    assert np.array_equal(blk, np.arange(41))


def test_planned_encode_equals_encode():
    """mtblx_encode_blocks_planned (the block cut's kept sums: no size pass, no look-back) writes
    exactly what mtblx_encode_blocks writes -- framed and unframed, the Writer's cut and arbitrary
    cuts inside the plan (0-record blocks included), intervals 1..40, blocks past the LDS buffer
    (assembled in HBM), cfg3 shards; a cut outside the plan is rejected per block."""
    enc = _enc()
    import torch
    from mtblx import synth
    rng = np.random.default_rng(65)

    def same(a, b, nb):
        for x, y in ((a.blk_off, b.blk_off), (a.blk_len, b.blk_len), (a.status, b.status)):
            assert torch.equal(x[:nb], y[:nb])
        assert torch.equal(a.totals, b.totals)
        t = int(a.totals[0].item())
        assert torch.equal(a.out[:t], b.out[:t])

    for bs, iv, n, kmax, vmax in [(4096, 16, 3000, 80, 200), (1024, 1, 800, 20, 10), (8192, 3, 2000, 300, 50),
                                  (65536, 40, 4000, 60, 120), (200_000, 16, 3000, 40, 150)]:
        recs = corpus.random_records(rng, n, 0, kmax, 0, vmax)
        d = enc.DeviceRecords.from_list(recs)
        blk, kept = enc.plan(d, bs, iv, keep=True)
        assert torch.equal(blk, enc.plan(d, bs, iv))
        for framed in (True, False):
            a = enc.encode_blocks(d, blk, iv, framed=framed)
            b = enc.encode_blocks(d, blk, iv, framed=framed, plan=kept)
            same(a, b, blk.numel() - 1)
        cuts = np.sort(rng.integers(0, n + 1, 30))
        arb = torch.tensor(np.concatenate([[0], cuts, [n]]), dtype=torch.int64, device="cuda")
        a = enc.encode_blocks(d, arb, iv, framed=True)
        b = enc.encode_blocks(d, arb, iv, framed=True, plan=kept)
        same(a, b, arb.numel() - 1)
    recs, _ = synth.cfg3_records_device(200_000, seed=4)
    sr = torch.tensor([0, 70_000, 200_000], dtype=torch.int64, device="cuda")
    blk, kept = enc.plan(recs, 65536, 16, shard_rec=sr, keep=True)
    same(enc.encode_blocks(recs, blk, 16), enc.encode_blocks(recs, blk, 16, plan=kept), blk.numel() - 1)
    # blocks of another cut that span the plan's shard start (record 70 000) share a
    # prefix there like mtblx_encode_blocks does (interval 16 and 7: the shard start in and out of
    # a restart phase)
    for iv in (16, 7):
        blk, kept = enc.plan(recs, 65536, iv, shard_rec=sr, keep=True)
        span = torch.tensor([0, 69_990, 70_013, 70_500, 200_000], dtype=torch.int64, device="cuda")
        same(enc.encode_blocks(recs, span, iv), enc.encode_blocks(recs, span, iv, plan=kept), span.numel() - 1)
    blk, kept = enc.plan(recs, 65536, 16, shard_rec=sr, keep=True)
    # a plan over the second shard only: blocks outside it are refused (UNSUPPORTED), the rest exact
    sr2 = torch.tensor([70_000, 200_000], dtype=torch.int64, device="cuda")
    blk2, kept2 = enc.plan(recs, 65536, 16, shard_rec=sr2, keep=True)
    mix = torch.cat([blk[:3], blk2])
    e = enc.encode_blocks(recs, mix, 16, plan=kept2)
    st = e.status.cpu().numpy()
    assert (st[:3] == 4).all() and (st[3:] == 0).all()
    # a LAST block outside the plan adds no bytes: totals[0] == the in-plan blocks' total
    sr3 = torch.tensor([0, 70_000], dtype=torch.int64, device="cuda")
    blk3, kept3 = enc.plan(recs, 65536, 16, shard_rec=sr3, keep=True)
    tail = torch.cat([blk3, torch.tensor([70_010], dtype=torch.int64, device="cuda")])
    e3 = enc.encode_blocks(recs, tail, 16, plan=kept3)
    ref = enc.encode_blocks(recs, blk3, 16, plan=kept3)
    assert int(e3.status[-1].item()) == 4 and int(e3.totals[0].item()) == int(ref.totals[0].item())

def test_cfg3_roundtrip_sample(oracle):
    """cfg3 scheme on the device: plan -> encode -> decode == the generated records; a sample of
    blocks against the oracle builder and decoder"""
    enc = _enc()
    import torch
    from mtblx import codec, synth
    recs, _ = synth.cfg3_records_device(300_000)
    blk = enc.plan(recs, 65536, 16, shard_rec=torch.tensor([0, 100_000, 300_000], dtype=torch.int64, device="cuda"))
    e = enc.encode_blocks(recs, blk, 16, framed=True)
    assert int(e.totals[1].item()) == 0
    assert int(e.blk_len.max().item()) <= 65536
    out = codec.decode_blocks(e.batch())
    torch.cuda.synchronize()
    nr, kb, vb, fl = out.totals_host()
    assert fl == 0 and nr == recs.n and (out.status[: out.nblk] == 0).all().item()
    assert torch.equal(out.keys[:kb], recs.keys) and torch.equal(out.vals[:vb], recs.vals)
    # key_end is block-relative u32: rebuild global ends and compare
    nrec = out.nrec[: out.nblk].to(torch.int64)
    blk_of = torch.repeat_interleave(torch.arange(out.nblk, device="cuda"), nrec)
    ke = out.key_base[: out.nblk][blk_of] + (out.key_end[:nr].to(torch.int64) & 0xFFFFFFFF)
    assert torch.equal(ke, recs.key_end)
    # oracle sample: a few blocks' bytes == oracle builder over the same records
    b = blk.cpu().numpy()
    ho = e.out.cpu().numpy()
    bo, bl = e.blk_off.cpu().numpy(), e.blk_len.cpu().numpy()
    keys, ke_h = recs.keys.cpu().numpy(), recs.key_end.cpu().numpy()
    vals, ve_h = recs.vals.cpu().numpy(), recs.val_end.cpu().numpy()
    for j in (0, 1, b.size // 2, b.size - 2):
        r0, r1 = int(b[j]), int(b[j + 1])
        rr = [(keys[(ke_h[r - 1] if r else 0): ke_h[r]].tobytes(), vals[(ve_h[r - 1] if r else 0): ve_h[r]].tobytes())
              for r in range(r0, r1)]
        assert ho[bo[j]: bo[j] + bl[j]].tobytes() == oracle.build_block(rr, 16)


def test_block_shapes_vs_writer(oracle):
    """k_encode at the edges of its paths: ~1000 and > 1024 entries per 64 KiB block, blocks
    over the LDS buffer (assembled in place in HBM), lengths around 76 KiB, interval-1 blocks
    of tiny entries, entry edges at every phase of 16 bytes -- byte for byte against the
    product Writer; the oracle reads every block back."""
    enc = _enc()
    rng = np.random.default_rng(64)
    cases = [
        (65536, 16, 9000, 0, 4, 0, 4),          # ~6 B entries: > 1024 per 64 KiB block
        (65536, 16, 3000, 0, 12, 0, 60),        # ~1000 entries per block: straddles the limit
        (131072, 4, 300, 0, 40, 0, 1500),       # 128 KiB blocks: in place in HBM
        (77000, 16, 400, 1, 30, 0, 900),        # block lengths around 76 KiB
        (1024, 1, 500, 0, 3, 0, 2),             # every entry a restart, blocks far under 16 B chunks
        (4096, 16, 2000, 0, 17, 15, 17),        # entry edges at every phase of the 16-byte chunks
    ]
    for bs, iv, n, kmin, kmax, vmin, vmax in cases:
        recs = corpus.random_records(rng, n, kmin, kmax, vmin, vmax)
        data, off, ln, nrec = _writer_file(recs, bs, iv)
        d = enc.DeviceRecords.from_list(recs)
        e = enc.encode_blocks(d, enc.plan(d, bs, iv), iv, framed=True)
        total = int(e.totals[0].item())
        assert int(e.totals[1].item()) == 0 and (e.status.cpu().numpy() == 0).all(), (bs, iv)
        idx_off = int(np.frombuffer(data[-512:-504], np.uint64)[0])
        assert total == idx_off, (bs, iv)
        assert e.out[:total].cpu().numpy().tobytes() == data[:idx_off], (bs, iv)
        orc = oracle.decode_blocks(e.out[:total].cpu().numpy(), off, ln)
        assert (orc.status == 0).all() and int(orc.nrec.sum()) == n
    # single records: empty key and value (the smallest block), one byte each
    for recs in ([(b"", b"")], [(b"k", b"v")], [(b"", b"x" * 70000)]):
        d = enc.DeviceRecords.from_list(recs)
        data, off, ln, _ = _writer_file(recs, 4096, 16)
        e = enc.encode_blocks(d, enc.plan(d, 4096, 16), 16, framed=True)
        total = int(e.totals[0].item())
        assert e.out[:total].cpu().numpy().tobytes() == data[:total]
