"""Deterministic synthetic workloads for BASELINE.json's configs.

cfg1  10 k keys "{:010}" / value "{:010}" * (1 + i % 8), 4 KiB blocks (examples/dump.rs plumbing)
cfg3  64 KiB blocks, key length 8 + k with P(k) ~ (k+1)^-1.1, k = 0..248 (mean ~40 B), keys =
      be64(c_i) || random tail (c_i = sum of gaps ~ U[1, 2^20)), 64 random value bytes,
      restart interval 16, seed 0x6d74626c03; generated on the device (cfg3_records_device)
cfg2  4 KiB blocks, 16 B keys = be64(c_i) || 8 random bytes with c_i = sum of gaps ~ U[1, 2^20)
      (strictly increasing, neighbours share ~5 B), 64 random value bytes, restart interval 16,
      CompressionType::None, seed 0x6d74626c02.
Files are produced by the product Writer (writer.py -> src/writer.rs semantics).
"""
from __future__ import annotations

import numpy as np

from .writer import Writer

SEED_CFG2 = 0x6D74626C02
SEED_CFG3 = 0x6D74626C03
SEED_CFG4 = 0x6D74626C04


def cfg1_records(n=10_000):
    for i in range(n):
        k = f"{i:010}"
        yield k.encode(), (k * (1 + i % 8)).encode()


def cfg2_arrays(nrec: int, seed: int = SEED_CFG2, key_tail: int = 8, val_len: int = 64, c0: int = 0):
    """keys (nrec*16 u8), values (nrec*64 u8) in record order; the key counter starts at c0."""
    rng = np.random.default_rng(seed)
    gaps = rng.integers(1, 1 << 20, nrec, dtype=np.uint64)
    c = np.cumsum(gaps, dtype=np.uint64) + np.uint64(c0)
    klen = 8 + key_tail
    keys = np.empty((nrec, klen), np.uint8)
    keys[:, :8] = c.astype(">u8").view(np.uint8).reshape(nrec, 8)
    keys[:, 8:] = rng.integers(0, 256, (nrec, key_tail), dtype=np.uint8)
    vals = rng.integers(0, 256, (nrec, val_len), dtype=np.uint8)
    return keys.reshape(-1), vals.reshape(-1), klen, val_len


def cfg2_keys(nrec: int, seed: int = SEED_CFG2, key_tail: int = 8, c0: int = 0):
    """the keys cfg2_arrays(nrec, seed, key_tail, c0=c0) draws, as an (nrec, 8 + key_tail) array,
    without its values (the same generator calls, in the same order, up to the key tails)"""
    rng = np.random.default_rng(seed)
    gaps = rng.integers(1, 1 << 20, nrec, dtype=np.uint64)
    c = np.cumsum(gaps, dtype=np.uint64) + np.uint64(c0)
    keys = np.empty((nrec, 8 + key_tail), np.uint8)
    keys[:, :8] = c.astype(">u8").view(np.uint8).reshape(nrec, 8)
    keys[:, 8:] = rng.integers(0, 256, (nrec, key_tail), dtype=np.uint8)
    return keys


def cfg2_file_nrec(nblocks: int, block_size: int = 4096) -> int:
    """the records cfg2_file generates (and writes) for `nblocks` blocks"""
    per_block = max(1, (block_size - 64) // 79)
    return int(nblocks * per_block * 1.02) + 64


def write_arrays(keys, vals, klen, vlen, block_size=4096, restart_interval=16):
    n = keys.size // klen
    w = Writer(block_size, restart_interval)
    ke = np.arange(1, n + 1, dtype=np.uint64) * np.uint64(klen)
    ve = np.arange(1, n + 1, dtype=np.uint64) * np.uint64(vlen)
    w.insert_batch(keys, ke, vals, ve)
    data = w.into_inner_np()
    off, ln = w.block_dir
    write_arrays.last_block_nrec = w.block_nrec
    return data, off, ln


def cfg2_file(nblocks: int = 100_000, block_size: int = 4096, seed: int = SEED_CFG2, c0: int = 0):
    """-> (file bytes as uint8 array, blk_off[nblocks], blk_len[nblocks]); exactly `nblocks` data blocks
    of the file are returned in the directory (the file may hold a few more).  c0: first key
    counter (shards of one key space: cfg2_shard)."""
    # ~51 records per 4 KiB block; generous estimate then trim the directory
    nrec = cfg2_file_nrec(nblocks, block_size)
    keys, vals, kl, vl = cfg2_arrays(nrec, seed, c0=c0)
    data, off, ln = write_arrays(keys, vals, kl, vl, block_size=block_size)
    while off.size < nblocks:  # extremely unlikely; extend
        nrec = int(nrec * 1.1)
        keys, vals, kl, vl = cfg2_arrays(nrec, seed, c0=c0)
        data, off, ln = write_arrays(keys, vals, kl, vl, block_size=block_size)
    cfg2_file.last_block_nrec = write_arrays.last_block_nrec[:nblocks].copy()
    return data, off[:nblocks].copy(), ln[:nblocks].copy()


SHARD_KEY_BITS = 56   # rank r's key counters start at r << 56 (a shard holds < 2^43 of them)


def cfg2_shard(rank: int, world: int, nblocks: int = 100_000, block_size: int = 4096):
    """Rank `rank`'s shard of a multi-GPU cfg2 workload: the key space is partitioned by rank
    (counters from rank << 56, seed SEED_CFG2 + rank), so the shards in rank order are one
    strictly increasing record stream -- the blocks of one logical file cut at block
    boundaries -- and every rank generates and decodes only its own `nblocks` blocks (weak
    scaling: per-GPU work fixed as the GPU count grows; no data-path collective)."""
    if not 0 <= rank < world:
        raise ValueError(f"rank {rank} outside world {world}")
    return cfg2_file(nblocks, block_size, seed=SEED_CFG2 + rank, c0=rank << SHARD_KEY_BITS)


def cfg3_key_len_probs():
    """P(key length = 8 + k) for k = 0..248, proportional to (k + 1)^-1.1"""
    w = (np.arange(249, dtype=np.float64) + 1.0) ** -1.1
    return w / w.sum()


def cfg3_records_device(nrec: int, seed: int = SEED_CFG3, c0: int = 0, device="cuda"):
    """cfg3 records on the device (torch as plumbing): -> (DeviceRecords, c_last).  c0 continues
    the key counter of a previous chunk so consecutive chunks stay strictly increasing."""
    import torch

    from .encode import DeviceRecords
    g = torch.Generator(device=device)
    g.manual_seed(int(seed) & ((1 << 63) - 1))
    probs = torch.tensor(cfg3_key_len_probs(), dtype=torch.float32, device=device)
    klen = torch.multinomial(probs, nrec, replacement=True, generator=g).to(torch.int64) + 8
    gaps = torch.randint(1, 1 << 20, (nrec,), generator=g, device=device, dtype=torch.int64)
    c = torch.cumsum(gaps, 0) + int(c0)
    key_end = torch.cumsum(klen, 0)
    total = int(key_end[-1].item())
    keys = torch.randint(0, 256, (total,), generator=g, device=device, dtype=torch.uint8)
    start = key_end - klen
    be = torch.stack([(c >> (8 * (7 - j))) & 0xFF for j in range(8)], 1).to(torch.uint8)   # big-endian c
    for j in range(8):
        keys[start + j] = be[:, j]
    vals = torch.randint(0, 256, (nrec * 64,), generator=g, device=device, dtype=torch.uint8)
    val_end = torch.arange(1, nrec + 1, device=device, dtype=torch.int64) * 64
    return DeviceRecords(keys, key_end, vals, val_end), int(c[-1].item())
