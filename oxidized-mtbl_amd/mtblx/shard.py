"""Block sharding across GPUs.

Blocks are independent units -- no decoder state crosses a block boundary
(/root/reference/src/block.rs:75-93, a fresh BlockIter per block in src/reader.rs:362-367) --
so a batch shards into contiguous ranges of the block directory with NO data-path
collective.  Cut points are byte-balanced: shard k starts at the first block whose
content prefix sum reaches k * total / world.  Every rank decodes its own range on its own
GPU; concatenating the shards' outputs in rank order gives exactly the unsharded output
(records keep the reference's order within and across blocks).
"""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np


def shard_cuts(blk_len: np.ndarray, world: int) -> np.ndarray:
    """world + 1 block indices; shard k = blocks [cuts[k], cuts[k+1])."""
    if world < 1:
        raise ValueError("world must be >= 1")
    ln = np.asarray(blk_len, dtype=np.uint64)
    n = ln.size
    incl = np.cumsum(ln, dtype=np.uint64)
    total = int(incl[-1]) if n else 0
    cuts = np.zeros(world + 1, np.int64)
    for k in range(1, world):
        target = (total * k) // world
        # first block whose exclusive prefix is >= target
        cuts[k] = int(np.searchsorted(incl, target, side="right")) if total else (n * k) // world
    cuts[world] = n
    return np.maximum.accumulate(np.minimum(cuts, n))


def shard_range(blk_len: np.ndarray, rank: int, world: int) -> tuple[int, int]:
    c = shard_cuts(blk_len, world)
    return int(c[rank]), int(c[rank + 1])


@dataclass
class ShardOutput:
    """Host copy of one shard's outputs in the include/mtblx.h layout."""
    nrec: np.ndarray
    status: np.ndarray
    key_end: np.ndarray
    val_end: np.ndarray
    keys: np.ndarray
    vals: np.ndarray


def concat_shards(parts: list) -> dict:
    """Rank-order concatenation: per-block arrays appended, bases recomputed as exclusive
    prefix sums over the whole batch; key_end/val_end are block-relative so they append
    unchanged."""
    nrec = np.concatenate([np.asarray(p.nrec, np.uint32) for p in parts])
    status = np.concatenate([np.asarray(p.status, np.int32) for p in parts])
    key_end = np.concatenate([np.asarray(p.key_end, np.uint32) for p in parts])
    val_end = np.concatenate([np.asarray(p.val_end, np.uint32) for p in parts])
    keys = np.concatenate([np.asarray(p.keys, np.uint8) for p in parts])
    vals = np.concatenate([np.asarray(p.vals, np.uint8) for p in parts])
    # block byte sizes from the block-relative ends (last record of each block)
    rec_base = np.zeros(nrec.size, np.uint64)
    rec_base[1:] = np.cumsum(nrec, dtype=np.uint64)[:-1]
    last = rec_base + nrec.astype(np.uint64) - 1
    has = nrec > 0
    kb = np.zeros(nrec.size, np.uint64)
    vb = np.zeros(nrec.size, np.uint64)
    kb[has] = key_end[last[has].astype(np.int64)]
    vb[has] = val_end[last[has].astype(np.int64)]
    key_base = np.zeros(nrec.size, np.uint64)
    val_base = np.zeros(nrec.size, np.uint64)
    key_base[1:] = np.cumsum(kb, dtype=np.uint64)[:-1]
    val_base[1:] = np.cumsum(vb, dtype=np.uint64)[:-1]
    return dict(nrec=nrec, status=status, rec_base=rec_base, key_base=key_base, val_base=val_base,
                key_end=key_end, val_end=val_end, keys=keys, vals=vals)
