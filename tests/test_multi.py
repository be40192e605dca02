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


def _bench():
    import importlib.util
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(root, "bench.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


def _bench_rank(rank, world, port, q):
    """bench.py's own rank path (init_ranks, the rank's cfg2 shard, rank_totals) on gloo, with
    the oracle's scan standing in for the device decode step"""
    import time
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), WORLD_SIZE=str(world), RANK=str(rank),
                      LOCAL_RANK=str(rank))
    import pyoracle
    bench = _bench()
    args = bench.parse_args(["--gpus", str(world), "--blocks", "120", "--steps", "3"])
    dist_, w, r, _ = bench.init_ranks(args, backend="gloo")
    assert (w, r) == (world, rank) and dist_ is not None
    data, off, ln = synth.cfg2_shard(r, w, args.blocks)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        d = pyoracle.decode_blocks(data, off, ln)
    el = time.perf_counter() - t0 + 0.05 * rank          # ranks finish at different times
    nrec = int(d.nrec.sum())
    tb, tr, tmax = bench.rank_totals(int(ln.sum()), nrec, el, dist_, device="cpu")
    first = bytes(d.records(0)[0][0])
    b = int(np.nonzero(d.nrec)[0][-1])
    last = bytes(d.records(b)[-1][0])
    edges = [None] * w
    dist_.all_gather_object(edges, (first, last, int(ln.sum()), nrec, el))   # checking only
    if r == 0:
        q.put((tb, tr, tmax, edges))
    dist_.barrier()
    dist_.destroy_process_group()


def test_gloo_bench_rank_path(oracle):
    """bench.py --gpus N runs N ranks that each decode their own shard; the line's
    value is the bytes of ALL ranks over the slowest rank's time.  Driven through bench.py's
    own functions on world_size-2 gloo (CPU); the shards continue one strictly increasing key
    space in rank order (one logical file cut at block boundaries)."""
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_bench_rank, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    tb, tr, tmax, edges = q.get(timeout=240)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert tb == sum(e[2] for e in edges) and tr == sum(e[3] for e in edges)
    assert tmax == max(e[4] for e in edges)
    assert edges[0][1] < edges[1][0]                      # rank 0's last key < rank 1's first key
    assert all(e[0] < e[1] for e in edges)


def test_bench_launch_and_world_checks(monkeypatch):
    """--gpus N outside torchrun re-launches through torch.distributed.run (N ranks); inside a
    launch, WORLD_SIZE must equal --gpus"""
    bench = _bench()
    args = bench.parse_args(["--gpus", "4", "--steps", "7"])
    cmd = bench.launch_command(["--gpus", "4", "--steps", "7"], 4, 29555)
    assert cmd[1:4] == ["-m", "torch.distributed.run", "--nnodes=1"] and "--nproc-per-node=4" in cmd
    assert "--master-addr" in cmd and cmd[cmd.index("--master-addr") + 1] == "127.0.0.1"
    assert cmd[-4:] == ["--gpus", "4", "--steps", "7"] and cmd[-5].endswith("bench.py")
    monkeypatch.setenv("WORLD_SIZE", "2")
    assert bench.maybe_launch(args, []) is None                 # already a rank: no re-launch
    with pytest.raises(SystemExit):
        bench.init_ranks(args, backend="gloo")                   # WORLD_SIZE 2 != --gpus 4
    monkeypatch.delenv("WORLD_SIZE")
    one = bench.parse_args([])
    assert one.gpus == 1 and bench.maybe_launch(one, []) is None


@pytest.mark.gpu
def test_bench_two_ranks_share_gpu():
    """the driver's N > 1 path end to end on a real GPU: `bench.py --gpus 2` relaunches itself
    through torch.distributed.run; with --share-gpu both ranks decode their shards on GPU 0 and
    the collectives go over gloo -- the JSON line must report both ranks' shards and records"""
    import json
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    cmd = [sys.executable, os.path.join(root, "bench.py"), "--gpus", "2", "--share-gpu", "--steps", "3",
           "--warmup", "1", "--blocks", "20000", "--no-crc", "--no-cpu-baseline"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=400, cwd=root)
    assert r.returncode == 0, "\n".join(ln for ln in r.stderr.splitlines() if ln.startswith("[rank"))[-4000:]
    line = [ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1]
    d = json.loads(line)
    assert d["n_gpus"] == 2 and d["value"] > 0
    assert "x2" in d["config"]["parallelism"] and "DIAGNOSTIC" in d["config"]["parallelism"]
