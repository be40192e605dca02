"""f1 on the matrix cores: k_crc32c_mfma (the default mtblx_crc32c_blocks kernel) against the
oracle's crc32c (crate crc32c 0.4, checked by tests/test_oracle.py against the CRC-32C check
value and the SURVEY §2.2 block CRCs) and against the VALU table kernel (MTBLX_CRC_KERNEL=lanes).

Shapes exercised: every length 0..600 (window and super-window edges, the < 4 B serial path, the
init fold straddling a window edge), blocks at buffer offsets 0..130 (the per-block path for
blocks that close to the buffer start), groups of 16 with one long block among short ones, blocks
above 256 KiB (the split pass: 16 columns of one block), block lengths that are not multiples of
anything, windows past the buffer end (bad = 1), and the framed check on a cfg2 file.
Reference: /root/reference/src/reader.rs:159-164 (the checksum Reader::block verifies)."""
import os

import numpy as np
import pytest

import corpus

pytestmark = pytest.mark.gpu


def _dev():
    from mtblx import codec
    codec._require_device()
    return codec


def _crc(codec, d, o, l, kernel, framed=False):
    import torch
    old = os.environ.get("MTBLX_CRC_KERNEL")
    os.environ["MTBLX_CRC_KERNEL"] = kernel
    try:
        batch = codec.DeviceBatch.from_host(d, o, l)
        crc, bad = codec.crc32c_blocks(batch, framed=framed)
        torch.cuda.synchronize()
    finally:
        if old is None:
            del os.environ["MTBLX_CRC_KERNEL"]
        else:
            os.environ["MTBLX_CRC_KERNEL"] = old
    return crc.cpu().numpy().view(np.uint32), (bad.cpu().numpy() if bad is not None else None)


def _expect(oracle, d, o, l):
    return np.array([oracle.crc32c(bytes(d[int(a): int(a) + int(n)])) for a, n in zip(o, l)], np.uint32)


@pytest.mark.parametrize("kernel", ["mfma", "lanes"])
def test_every_length(oracle, kernel):
    codec = _dev()
    rng = np.random.default_rng(41)
    blocks = [bytes(rng.integers(0, 256, n, dtype=np.uint8)) for n in range(0, 601)]
    order = rng.permutation(len(blocks))   # groups of 16 mix short and long blocks
    d, o, l = corpus.pack([blocks[i] for i in order], rng=rng, lead=200)
    got, _ = _crc(codec, d, o, l, kernel)
    exp = _expect(oracle, d, o, l)
    assert np.array_equal(got, exp), np.nonzero(got != exp)[0][:10]


@pytest.mark.parametrize("kernel", ["mfma", "lanes"])
def test_near_buffer_start_and_end(oracle, kernel):
    """blocks at offsets 0..130 (loads must not start before the buffer) and a window that runs
    past the buffer end (the reference's slice panics: bad = 1, crc 0)"""
    codec = _dev()
    rng = np.random.default_rng(42)
    data = rng.integers(0, 256, 9000, dtype=np.uint8)
    off, ln = [], []
    for a in list(range(0, 131, 3)) + [127, 128, 129]:
        for n in (4, 5, 100, 127, 128, 129, 300, 4000):
            off.append(a)
            ln.append(n)
    off += [8990, 100, 8000]
    ln += [20, 0, 1000]                                   # the first runs past the end
    o, l = np.array(off, np.uint64), np.array(ln, np.uint32)
    got, bad = _crc(codec, data, o, l, kernel, framed=True)
    ok = (o + l) <= data.size
    exp = _expect(oracle, data, o, l)
    assert np.array_equal(got[ok], exp[ok])
    assert np.array_equal(bad[~ok], np.ones((~ok).sum(), np.uint8))
    assert (got[~ok] == 0).all()


@pytest.mark.parametrize("kernel", ["mfma", "lanes"])
def test_long_blocks_split_pass(oracle, kernel):
    """blocks above 256 KiB (one wave, 16 columns, super-window shifts past 16) beside short ones"""
    codec = _dev()
    rng = np.random.default_rng(43)
    sizes = [300_000, 5, 4096, 262_144, 262_145, 1_100_001, 70_000, 3, 65_536, 4_200_000]
    blocks = [bytes(rng.integers(0, 256, n, dtype=np.uint8)) for n in sizes]
    d, o, l = corpus.pack(blocks, rng=rng, lead=300)
    got, _ = _crc(codec, d, o, l, kernel)
    exp = _expect(oracle, d, o, l)
    assert np.array_equal(got, exp), np.nonzero(got != exp)[0]


def test_cfg2_framed_both_kernels(oracle):
    codec = _dev()
    from mtblx import synth
    data, off, ln = synth.cfg2_file(5000)
    d2 = data.copy()
    for b in (0, 15, 16, 4999):
        d2[int(off[b]) - 3] ^= 0x10
    d2[int(off[2000]) + 7] ^= 0x80
    exp = _expect(oracle, d2, off, ln)
    for kernel in ("mfma", "lanes"):
        got, bad = _crc(codec, d2, off, ln, kernel, framed=True)
        assert np.array_equal(got, exp)
        assert sorted(np.nonzero(bad)[0].tolist()) == [0, 15, 16, 2000, 4999]
