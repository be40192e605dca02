"""CPU tests of the full-size parity checker (oracle_check_writer_blocks) that
tests/test_cfg3_oracle_gpu.py runs over every cfg3 block: fed the product host Writer's output
(byte-identical to the oracle Writer, pinned by the golden files) it must report every block and
record equal, and it must catch a changed content byte, a changed checksum, a wrong cut and a
record that differs from the block (positive controls)."""
import numpy as np

from mtblx.writer import Writer


def _records(n, seed):
    rng = np.random.default_rng(seed)
    klen = 8 + rng.zipf(1.6, n).clip(1, 200)
    c = np.cumsum(rng.integers(1, 1 << 20, n, dtype=np.uint64))
    key_end = np.cumsum(klen).astype(np.uint64)
    keys = rng.integers(0, 256, int(key_end[-1]), dtype=np.uint8)
    start = key_end - klen.astype(np.uint64)
    be = c.astype(">u8").view(np.uint8).reshape(n, 8)
    for j in range(8):
        keys[(start + np.uint64(j)).astype(np.int64)] = be[:, j]
    vals = rng.integers(0, 256, 64 * n, dtype=np.uint8)
    val_end = np.arange(1, n + 1, dtype=np.uint64) * np.uint64(64)
    return keys, key_end, vals, val_end


def _device_like(keys, key_end, vals, val_end, shard_rec, block_size, iv):
    """framed data blocks of one independent Writer per shard, back to back (the device encode's
    output layout): -> (bytes, content offsets, lengths, blk_rec)"""
    parts, offs, lens, brec, base = [], [], [], [0], 0
    for s in range(len(shard_rec) - 1):
        r0, r1 = int(shard_rec[s]), int(shard_rec[s + 1])
        k0 = int(key_end[r0 - 1]) if r0 else 0
        v0 = int(val_end[r0 - 1]) if r0 else 0
        w = Writer(block_size, iv)
        w.insert_batch(keys[k0:int(key_end[r1 - 1])], key_end[r0:r1] - np.uint64(k0),
                       vals[v0:int(val_end[r1 - 1])], val_end[r0:r1] - np.uint64(v0))
        f = w.into_inner_np()
        off, ln = w.block_dir
        data_end = int(off[-1]) + int(ln[-1])
        parts.append(f[:data_end])
        offs.append(off.astype(np.uint64) + np.uint64(base))
        lens.append(ln)
        brec.extend((r0 + np.cumsum(w.block_nrec.astype(np.int64))).tolist())
        base += data_end
    return (np.concatenate(parts), np.concatenate(offs), np.concatenate(lens).astype(np.uint32),
            np.array(brec, np.int64))


def test_checker_accepts_writer_output_and_catches_changes(oracle):
    n = 6000
    keys, key_end, vals, val_end = _records(n, 0x63686b)
    shard_rec = np.array([0, 1, 1700, 4321, n], np.int64)      # a one-record shard included
    f, off, ln, brec = _device_like(keys, key_end, vals, val_end, shard_rec, 8192, 16)
    nb = off.size
    r = oracle.check_writer_blocks(f, off, ln, brec, keys, key_end, vals, val_end, shard_rec, 8192, 16, 4)
    assert r == dict(blocks_equal=nb, blocks=nb, records_equal=n, records=n, first_bad_block=None,
                     shards_misaligned=0), r

    b = nb // 2
    g = f.copy()
    g[int(off[b]) + 7] ^= 1                                      # a content byte
    r = oracle.check_writer_blocks(g, off, ln, brec, keys, key_end, vals, val_end, shard_rec, 8192, 16, 4)
    assert r["blocks_equal"] == nb - 1 and r["first_bad_block"] == b

    g = f.copy()
    g[int(off[3]) - 2] ^= 0x40                                   # the stored crc32c
    r = oracle.check_writer_blocks(g, off, ln, brec, keys, key_end, vals, val_end, shard_rec, 8192, 16, 4)
    assert r["blocks_equal"] == nb - 1 and r["records_equal"] == n and r["first_bad_block"] == 3

    v2 = vals.copy()
    v2[64 * int(brec[5]) + 3] ^= 0x10                            # the input record, not the block
    r = oracle.check_writer_blocks(f, off, ln, brec, keys, key_end, v2, val_end, shard_rec, 8192, 16, 4)
    assert r["records_equal"] == n - 1 and r["blocks_equal"] < nb

    b2 = brec.copy()
    b2[4] += 1                                                   # a cut that is not the Writer's
    r = oracle.check_writer_blocks(f, off, ln, b2, keys, key_end, vals, val_end, shard_rec, 8192, 16, 4)
    assert r["records_equal"] < n and r["first_bad_block"] is not None

    # the device truncates a chunk's cut to whole blocks: the last shard ends early
    cut = int(brec[nb - 3])
    r = oracle.check_writer_blocks(f, off[:nb - 3], ln[:nb - 3], brec[:nb - 2], keys, key_end, vals, val_end,
                                   shard_rec, 8192, 16, 4)
    assert r == dict(blocks_equal=nb - 3, blocks=nb - 3, records_equal=cut, records=cut, first_bad_block=None,
                     shards_misaligned=0), r
