"""Seeded block corpora shared by the CPU and GPU parity tests.

Blocks are built with the ORACLE BlockBuilder (src/block_builder.rs restated), then some
are mutated so every reference outcome appears: OK on the regular fast path, OK on the
irregular path (restart quirks, non-canonical varints, shared > previous length within
Vec capacity), INVALID_BLOCK, CORRUPT with a prefix of yielded records, and LOOP.
"""
from __future__ import annotations

import json
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))


def quirk_blocks():
    q = json.load(open(os.path.join(HERE, "golden", "quirk_blocks.json")))
    return [(d["name"], bytes.fromhex(d["block"]), d) for d in q]


def random_records(rng, n, kmin=0, kmax=40, vmin=0, vmax=80, prefix_bias=True):
    """n strictly increasing random keys (shared prefixes common) + random values."""
    keys = set()
    base = rng.integers(0, 256, kmax + 8, dtype=np.uint8).tobytes()
    while len(keys) < n:
        kl = int(rng.integers(kmin, kmax + 1))
        if prefix_bias and kl > 0 and rng.random() < 0.7:
            p = int(rng.integers(0, kl + 1))
            k = base[:p] + rng.integers(0, 256, kl - p, dtype=np.uint8).tobytes()
        else:
            k = rng.integers(0, 256, kl, dtype=np.uint8).tobytes()
        keys.add(k)
    keys = sorted(keys)
    vals = [rng.integers(0, 256, int(rng.integers(vmin, vmax + 1)), dtype=np.uint8).tobytes() for _ in range(n)]
    return list(zip(keys, vals))


def builder_blocks(oracle, seed=1, count=200, max_bytes=7000):
    """Valid blocks from the BlockBuilder with random shapes (restart interval 1..40)."""
    rng = np.random.default_rng(seed)
    blocks = []
    while len(blocks) < count:
        iv = int(rng.choice([1, 2, 3, 8, 16, 16, 16, 17, 32, 40]))
        kmax = int(rng.choice([4, 16, 40, 120, 300]))
        vmax = int(rng.choice([0, 8, 64, 200]))
        n = int(rng.integers(0, 120))
        recs = random_records(rng, n, 0, kmax, 0, vmax)
        b = oracle.build_block(recs, restart_interval=iv)
        if len(b) <= max_bytes:
            blocks.append(b)
    return blocks


def mutate(rng, block: bytes) -> bytes:
    b = bytearray(block)
    if not b:
        return bytes(b)
    kind = int(rng.integers(0, 7))
    if kind == 0:      # flip a byte anywhere
        i = int(rng.integers(0, len(b)))
        b[i] ^= int(rng.integers(1, 256))
    elif kind == 1:    # corrupt the restart count
        if len(b) >= 4:
            b[-4:] = int(rng.integers(0, 1 << 32)).to_bytes(4, "little")
    elif kind == 2:    # corrupt a restart point
        if len(b) >= 8:
            n = int.from_bytes(b[-4:], "little")
            if 0 < n < len(b) // 4:
                j = len(b) - 4 - 4 * (n - int(rng.integers(0, n)))
                b[j:j + 4] = int(rng.integers(0, len(b) + 8)).to_bytes(4, "little")
    elif kind == 3:    # set a high bit in an early header byte (slow path)
        i = int(rng.integers(0, min(len(b), 64)))
        b[i] |= 0x80
    elif kind == 4:    # truncate the entry region
        if len(b) > 12:
            cut = int(rng.integers(1, min(8, len(b) - 8)))
            n = bytes(b[-4:])
            rs = bytes(b[-8:-4])
            b = b[: len(b) - 8 - cut] + rs + n
    elif kind == 5:    # bump a shared value
        i = int(rng.integers(0, min(len(b), 200)))
        b[i] = (b[i] + int(rng.integers(1, 8))) & 0x7F
    else:              # random length
        b = b[: int(rng.integers(0, len(b) + 1))]
    return bytes(b)


def mutated_blocks(oracle, seed=2, count=600):
    rng = np.random.default_rng(seed)
    base = builder_blocks(oracle, seed=seed + 100, count=120, max_bytes=4000)
    out = []
    for i in range(count):
        blk = base[i % len(base)]
        for _ in range(int(rng.integers(1, 3))):
            blk = mutate(rng, blk)
        out.append(blk)
    return out


def pack(blocks, align=1, lead=0, rng=None):
    """Concatenate blocks into one buffer with optional gaps (unaligned offsets)."""
    parts, off, ln = [], [], []
    pos = 0
    if lead:
        parts.append(b"\xAB" * lead)
        pos += lead
    for b in blocks:
        gap = int(rng.integers(0, 9)) if rng is not None else 0
        if gap:
            parts.append(bytes(rng.integers(0, 256, gap, dtype=np.uint8)))
            pos += gap
        off.append(pos)
        ln.append(len(b))
        parts.append(b)
        pos += len(b)
    data = np.frombuffer(b"".join(parts) or b"\0", np.uint8).copy()
    return data, np.array(off, np.uint64), np.array(ln, np.uint32)


# ---------------- FormatV1 files (src/metadata.rs:29-33, src/reader.rs:54-56,146-148) ----------------
MAGIC_V1 = 0x77846676


def to_v1(data: bytes, restart_interval=16) -> bytes:
    """Re-frame a FormatV2 file (an oracle / product Writer output) as FormatV1: every block's
    varint64 length becomes a u32 LE length (src/reader.rs:146-148; index: :54-56), the stored
    checksum and content stay (the CRC covers the stored content), the index block is rebuilt
    with the same separators and the new block offsets as varint64 values (the BlockBuilder
    the Writer uses for its index, src/writer.rs:72,136,160), and the footer gets the new
    offsets / byte counts and the V1 magic (src/metadata.rs:29-33, src/lib.rs:17-20).
    The reference only writes V2 (src/writer.rs:215); its reader takes both."""
    import pyoracle as o
    data = bytes(data)
    meta = [int.from_bytes(data[len(data) - 512 + 8 * i: len(data) - 504 + 8 * i], "little") for i in range(9)]
    out = bytearray()
    entries = []
    for sep, val in o.index_records(data):
        off, _ = o.varint_decode64(val)
        n, ll = o.varint_decode64(data[off: off + 10])
        entries.append((sep, o.varint_encode64(len(out))))
        out += n.to_bytes(4, "little") + data[off + ll: off + ll + 4 + n]
    nbytes_data = len(out)
    ib = o.build_block(entries, restart_interval)
    idx_off = len(out)
    out += len(ib).to_bytes(4, "little") + o.crc32c(ib).to_bytes(4, "little") + ib
    meta[0], meta[5], meta[6] = idx_off, nbytes_data, len(out) - idx_off
    footer = b"".join(m.to_bytes(8, "little") for m in meta)
    footer += b"\0" * (508 - len(footer)) + MAGIC_V1.to_bytes(4, "little")
    return bytes(out) + footer


def v1_frames(data: bytes):
    """(frame offset, content length) of every block of a V1 file, index block last"""
    import pyoracle as o
    idx_off = int.from_bytes(data[len(data) - 512: len(data) - 504], "little")
    n = int.from_bytes(data[idx_off: idx_off + 4], "little")
    st, recs = o.decode_block(data[idx_off + 8: idx_off + 8 + n])
    frames = []
    for _, val in recs:
        off, _ = o.varint_decode64(val)
        frames.append((off, int.from_bytes(data[off: off + 4], "little")))
    return frames + [(idx_off, n)]
