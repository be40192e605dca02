"""BASELINE configs[3] (cfg4) block shapes against the oracle, bit for bit.

cfg4 = the cfg2 key/value scheme (16 B keys, 64 B values, restart interval 16) written with
4, 16 and 64 KiB blocks, decoded as one sharded directory.  These tests pin exactly those
shapes at oracle-checkable sizes (a few hundred blocks per leg):
- each leg alone (PipeSmall for 4 / 16 KiB, PipeLarge for 64 KiB);
- the three legs as ONE mixed batch in a single mtblx_decode_blocks call;
- that mixed directory cut into 2 byte-balanced shards with mtblx.shard.shard_cuts (the cut
  bench.py --config cfg4 uses), each shard decoded on its own and concatenated in rank order,
  equal to the unsharded decode.
"""
import numpy as np
import pytest

from mtblx import shard, synth

pytestmark = pytest.mark.gpu

LEGS = ((4096, 600), (16384, 300), (65536, 120))


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


def _same(dev, orc):
    for k in ("status", "nrec", "rec_base", "key_base", "val_base", "key_end", "val_end", "keys", "vals"):
        a, b = getattr(dev, k), getattr(orc, k)
        assert a.shape == b.shape and np.array_equal(a, b), k
    assert dev.totals[3] == 0


def _leg(bs, nblk, li):
    return synth.cfg2_file(nblk, block_size=bs, seed=synth.SEED_CFG4 + li)


def _mixed():
    """the three legs' files back to back in one buffer, one directory"""
    parts, offs, lens, base = [], [], [], 0
    for li, (bs, nb) in enumerate(LEGS):
        d, o, l_ = _leg(bs, nb, li)
        parts.append(d)
        offs.append(o.astype(np.uint64) + np.uint64(base))
        lens.append(l_)
        base += d.size
    return np.concatenate(parts), np.concatenate(offs), np.concatenate(lens)


@pytest.mark.parametrize("li", range(len(LEGS)))
def test_cfg4_leg_vs_oracle(oracle, li):
    bs, nb = LEGS[li]
    data, off, ln = _leg(bs, nb, li)
    assert int(ln.max()) > bs - 200 and off.size == nb
    orc = oracle.decode_blocks(data, off, ln)
    assert (orc.status == 0).all() and int(orc.nrec.sum()) > 0
    # interval 16: restarts every 16 records
    assert int(orc.nrec.max()) > 16
    _same(_decode(data, off, ln), orc)


def test_cfg4_mixed_batch_one_call(oracle):
    data, off, ln = _mixed()
    orc = oracle.decode_blocks(data, off, ln)
    assert (orc.status == 0).all()
    _same(_decode(data, off, ln), orc)


def test_cfg4_two_shards_concat(oracle):
    data, off, ln = _mixed()
    full = _decode(data, off, ln)
    cuts = shard.shard_cuts(ln, 2)
    assert 0 < cuts[1] < off.size
    parts = []
    for r in range(2):
        b0, b1 = int(cuts[r]), int(cuts[r + 1])
        h = _decode(data, off[b0:b1], ln[b0:b1])
        parts.append(shard.ShardOutput(h.nrec, h.status, h.key_end, h.val_end, h.keys, h.vals))
    cat = shard.concat_shards(parts)
    for k in ("nrec", "status", "rec_base", "key_base", "val_base", "key_end", "val_end", "keys", "vals"):
        assert np.array_equal(cat[k], getattr(full, k)), k
    # byte-balanced: the shards hold about half of the block bytes each
    b = [int(ln[int(cuts[r]):int(cuts[r + 1])].sum()) for r in range(2)]
    assert abs(b[0] - b[1]) <= 2 * int(ln.max())
