"""Emitting block seek on one block of GiBs (src/block.rs:25-42, :106-213): the values moved
by the seeking wave (mtblx_block_seek_batch) against the round-5 form (mtblx_block_seek_batch_ex
records each value's content offset, mtblx_copy_ranges moves them with the whole grid).

The block is assembled here by hand (BlockBuilder layout: shared=0 headers, restarts [0], count
1; src/block_builder.rs:69-77, :85-104), so no oracle is involved; the two forms must agree byte
for byte.  Prints one JSON line: ms per seek (HIP events) for each form and the value bytes."""
import argparse
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "oxidized-mtbl_amd"))
from mtblx import iterator  # noqa: E402


def varint(v: int) -> bytes:
    out = bytearray()
    while v >= 128:
        out.append((v & 127) | 128)
        v >>= 7
    out.append(v)
    return bytes(out)


def block(vlens, dev):
    """records k000.. with values of the given lengths (a byte ramp each), built on the device"""
    parts, spans = [], []
    pos = 0
    for i, vl in enumerate(vlens):
        k = b"k%05d" % i
        h = varint(0) + varint(len(k)) + varint(vl) + k
        parts.append(torch.tensor(list(h), dtype=torch.uint8, device=dev))
        pos += len(h)
        spans.append((pos, vl))
        parts.append((torch.arange(vl, device=dev, dtype=torch.int64) * (i + 7) % 251).to(torch.uint8))
        pos += vl
    parts.append(torch.tensor(list((0).to_bytes(4, "little") + (1).to_bytes(4, "little")), dtype=torch.uint8, device=dev))
    return torch.cat(parts)


def timed(fn, reps):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        r = fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps, r


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mib", type=int, default=1024, help="value bytes in the block, MiB")
    ap.add_argument("--reps", type=int, default=3)
    a = ap.parse_args()
    dev = torch.device("cuda")
    tot = a.mib << 20
    vl = [5, tot // 2 - 3, 17, tot // 2 - 19]
    blk = block(vl, dev)
    content = (blk, 0, int(blk.numel()))
    grid_ms, g = timed(lambda: iterator.block_seek(content, None, small_caps=True), a.reps)
    old = iterator._BIG_BLOCK
    iterator._BIG_BLOCK = 1 << 62   # the seeking wave moves the values (the pre-round-5 form)
    try:
        wave_ms, w = timed(lambda: iterator.block_seek(content, None), a.reps)
    finally:
        iterator._BIG_BLOCK = old
    same = (g.nrec == w.nrec == len(vl) and torch.equal(g.keys, w.keys) and torch.equal(g.vals, w.vals)
            and torch.equal(g.val_end, w.val_end))
    vb = int(g.val_end[-1].item())
    print(json.dumps({"probe": "block seek of one block of GiBs", "block_bytes": int(blk.numel()), "value_bytes": vb,
                      "wave_ms": round(wave_ms, 3), "grid_ms": round(grid_ms, 3),
                      "wave_GBs": round(vb / wave_ms / 1e6, 1), "grid_GBs": round(vb / grid_ms / 1e6, 1),
                      "identical": bool(same)}))
    if not same:
        sys.exit(1)


if __name__ == "__main__":
    main()
