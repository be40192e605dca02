"""N>1 path: block sharding with no data-path collective.

CPU tests run world_size-2 `gloo` process groups: each rank decodes its byte-balanced shard
with the oracle (the checker; the GPU product path is exercised per rank by bench.py under
torchrun), shards are gathered only to CHECK, and the rank-order concatenation must equal
the unsharded decode bit for bit.  The GPU test decodes two shards with the HIP path on one
device and compares the concatenation with a single-batch device decode.
"""
import os
import socket

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

from mtblx import shard, synth


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_shard_cuts_cover_and_balance():
    rng = np.random.default_rng(5)
    ln = rng.integers(1, 70000, 1000).astype(np.uint32)
    for world in (1, 2, 3, 4, 8):
        c = shard.shard_cuts(ln, world)
        assert c[0] == 0 and c[-1] == ln.size and np.all(np.diff(c) >= 0)
        sizes = [int(ln[c[k]:c[k + 1]].sum()) for k in range(world)]
        assert sum(sizes) == int(ln.sum())
        assert max(sizes) - min(sizes) <= 2 * int(ln.max())   # byte-balanced to within a block or two
    assert list(shard.shard_cuts(np.zeros(0, np.uint32), 2)) == [0, 0, 0]
    assert list(shard.shard_cuts(np.array([5], np.uint32), 4))[-1] == 1


def _records(d):
    return [d.records(b) for b in range(d.nrec.size)]


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import pyoracle
    data, off, ln = synth.cfg2_file(300)
    b0, b1 = shard.shard_range(ln, rank, world)
    d = pyoracle.decode_blocks(data, off[b0:b1], ln[b0:b1])
    part = shard.ShardOutput(d.nrec, d.status, d.key_end, d.val_end, d.keys, d.vals)
    parts = [None] * world
    dist.all_gather_object(parts, part)   # checking only; the product path has no collective
    if rank == 0:
        full = pyoracle.decode_blocks(data, off, ln)
        cat = shard.concat_shards(parts)
        ok = all(np.array_equal(cat[k], getattr(full, k)) for k in
                 ("nrec", "status", "rec_base", "key_base", "val_base", "key_end", "val_end", "keys", "vals"))
        q.put((ok, int(cat["nrec"].sum()), [int(p.nrec.size) for p in parts]))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2])
def test_gloo_sharded_decode_equals_unsharded(oracle, world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = q.get(timeout=240)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    ok, nrec, sizes = res
    assert ok and nrec > 0 and sum(sizes) == 300 and min(sizes) > 0


@pytest.mark.gpu
def test_gpu_two_shards_concat_equals_single_batch():
    from mtblx import codec
    data, off, ln = synth.cfg2_file(2000)
    full = codec.decode_blocks(codec.DeviceBatch.from_host(data, off, ln)).to_host()
    parts = []
    for r in range(2):
        b0, b1 = shard.shard_range(ln, r, 2)
        h = codec.decode_blocks(codec.DeviceBatch.from_host(data, off[b0:b1], ln[b0:b1])).to_host()
        parts.append(shard.ShardOutput(h.nrec, h.status, h.key_end, h.val_end, h.keys, h.vals))
    cat = shard.concat_shards(parts)
    for k in ("nrec", "status", "rec_base", "key_base", "val_base", "key_end", "val_end", "keys", "vals"):
        assert np.array_equal(cat[k], getattr(full, k)), k
