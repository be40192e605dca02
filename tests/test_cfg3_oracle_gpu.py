"""cfg3 (BASELINE configs[2]) with CPU-oracle parity on EVERY block ("bit-exact
decode(encode(x)) == x, with CPU-oracle parity on every block (chunked)").

The same chunks as bench.py's cfg3 leg (rank 0: seeds SEED_CFG3 + chunk, chained key counters, 64
Writer shards per chunk, the cut truncated to whole blocks): device block cut
(mtblx_encode_plan_keep) -> planned encode (mtblx_encode_blocks_planned, framed) -> device decode
(mtblx_decode_blocks).  Per chunk, outside any timed region:
  - on the device: every decoded record == the generated record (keys, values, key END offsets);
  - on the host, 16 threads: the oracle Writer (src/writer.rs:112-237 + src/block_builder.rs:49-104,
    oracle/mtbl_oracle.c) over each shard's records == the device's framed blocks, frame by frame
    (length varint, crc32c, content), and the restated decode (src/block.rs:119-238) of every
    device block == the generated records.

Default size: 20 000 blocks (the -m gpu suite).  MTBLX_CFG3_BLOCKS=1000000 runs the full config
(~65 GB of blocks in 10 chunks); MTBLX_CFG3_LOG appends one line per chunk to a file.
"""
import json
import os
import time

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _threads():
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else os.cpu_count()
    return max(1, min(16, n or 1))


def test_cfg3_every_block_vs_oracle(oracle):
    from mtblx import codec, encode, synth
    total = int(os.environ.get("MTBLX_CFG3_BLOCKS", "20000"))
    per_chunk = int(os.environ.get("MTBLX_CFG3_CHUNK", "100000"))
    logp = os.environ.get("MTBLX_CFG3_LOG")
    nth = _threads()
    s = torch.cuda.Stream()
    acc = dict(blocks=0, blocks_equal=0, records=0, records_equal=0, device_records_equal=0, block_bytes=0,
               shards_misaligned=0, chunks=0, oracle_s=0.0, d2h_s=0.0)
    done, ci, c0 = 0, 0, 0
    while done < total:
        want = min(per_chunk, total - done)
        nrec = int(want * 640 * 1.03) + 1024                      # bench.py run_cfg3's sizing
        recs, c_last = synth.cfg3_records_device(nrec, seed=synth.SEED_CFG3 + ci, c0=c0)
        c0 = c_last
        cuts = torch.linspace(0, nrec, 65, device="cuda").to(torch.int64)
        blk, kept = encode.plan(recs, 65536, 16, shard_rec=cuts, keep=True)
        blk = blk[: want + 1].contiguous()
        nb = int(blk.numel()) - 1
        bufs = encode.EncodeBuffers(recs, nb)
        with torch.cuda.stream(s):
            e = encode.encode_into(recs, blk, bufs, 16, True, s, plan=kept)
        torch.cuda.synchronize()
        e.check()
        assert int(e.totals[1].item()) == 0 and bool((e.status == 0).all().item())
        batch = e.batch()
        with torch.cuda.stream(s):
            ws = codec.Workspace(nb)
            probe = codec.DecodedBlocks(nb, 0, 0, 0)
            codec.count_blocks(batch, probe, ws, s)
        torch.cuda.synchronize()
        nr, kb, vb, _ = probe.totals_host()
        with torch.cuda.stream(s):
            out = codec.DecodedBlocks(nb, nr, kb, vb)
            codec.decode_into(batch, out, ws, s)
        torch.cuda.synchronize()
        r_used = int(blk[-1].item())
        ok = nr == r_used and kb == int(recs.key_end[r_used - 1].item()) and vb == 64 * r_used
        ok = ok and out.totals_host()[3] == 0 and bool((out.status[:nb] == 0).all().item())
        ok = ok and torch.equal(out.keys[:kb], recs.keys[:kb]) and torch.equal(out.vals[:vb], recs.vals[:vb])
        nrb = out.nrec[:nb].to(torch.int64)
        blk_of = torch.repeat_interleave(torch.arange(nb, device="cuda"), nrb)
        ke = out.key_base[:nb][blk_of] + (out.key_end[:nr].to(torch.int64) & 0xFFFFFFFF)
        ok = ok and torch.equal(ke, recs.key_end[:nr]) and torch.equal(torch.cumsum(nrb, 0), blk[1:] - blk[0])
        acc["device_records_equal"] += nr if ok else 0
        # to the host: the framed blocks, the directory, the cut and the input records
        t0 = time.perf_counter()
        file_len = int(e.blk_off[nb - 1].item()) + int(e.blk_len[nb - 1].item())
        h_file = e.out[:file_len].cpu().numpy()
        h_off = e.blk_off.cpu().numpy().astype(np.uint64)
        h_len = e.blk_len.cpu().numpy().view(np.uint32)
        h_blk = blk.cpu().numpy()
        h_keys = recs.keys[:int(recs.key_end[r_used - 1].item())].cpu().numpy()
        h_ke = recs.key_end[:r_used].cpu().numpy().view(np.uint64)
        h_vals = recs.vals[:64 * r_used].cpu().numpy()
        h_ve = recs.val_end[:r_used].cpu().numpy().view(np.uint64)
        h_cuts = cuts.cpu().numpy()
        acc["d2h_s"] += time.perf_counter() - t0
        t0 = time.perf_counter()
        r = oracle.check_writer_blocks(h_file, h_off, h_len, h_blk, h_keys, h_ke, h_vals, h_ve, h_cuts, 65536, 16, nth)
        dt = time.perf_counter() - t0
        acc["oracle_s"] += dt
        for k in ("blocks", "blocks_equal", "records", "records_equal", "shards_misaligned"):
            acc[k] += r[k]
        acc["block_bytes"] += int(h_len.astype(np.int64).sum())
        acc["chunks"] += 1
        line = (f"cfg3 chunk {ci + 1}: {nb} blocks, device round trip {'ok' if ok else 'FAILED'}; oracle-equal "
                f"blocks {r['blocks_equal']} / {r['blocks']}, records {r['records_equal']} / {r['records']}, "
                f"first bad {r['first_bad_block']}, misaligned shards {r['shards_misaligned']} ({dt:.1f} s, {nth} threads)")
        print(line, flush=True)
        if logp:
            with open(logp, "a") as fh:
                fh.write(line + "\n")
        assert ok, line
        assert r["blocks_equal"] == nb == r["blocks"] and r["records_equal"] == r_used == r["records"], line
        assert r["shards_misaligned"] == 0, line
        done += nb
        ci += 1
        del recs, blk, kept, bufs, e, batch, ws, probe, out, h_file, h_keys, h_vals, blk_of, ke, nrb
        torch.cuda.empty_cache()
    summary = (f"oracle-equal blocks {acc['blocks_equal']} / {acc['blocks']}, records {acc['records_equal']} / "
               f"{acc['records']} (device round trip: {acc['device_records_equal']} records), "
               f"{acc['block_bytes']} block bytes, {acc['chunks']} chunks; oracle {acc['oracle_s']:.1f} s on {nth} "
               f"threads, D2H {acc['d2h_s']:.1f} s")
    print(summary, flush=True)
    if logp:
        with open(logp, "a") as fh:
            fh.write(summary + "\n" + json.dumps(acc) + "\n")
    assert acc["blocks_equal"] == acc["blocks"] == total
