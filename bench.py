#!/usr/bin/env python3
"""bench.py — device-resident mtbl block-decode throughput on MI355X.

Metric (BASELINE.json): "KV records/s + GiB/s of block bytes decoded, device-resident,
1/2/4/8 GPU".  Workload (N=1): BASELINE configs[1] = cfg2, 100 k data blocks of 4 KiB,
16 B keys / 64 B values, restart interval 16, CompressionType::None,
written by the product Writer from a seeded generator (synthetic data).

A step = one full decode of the resident batch through the C ABI (mtblx_decode_blocks:
one single-pass k_decode_pipe launch for blocks <= 48 KiB, k_decode_tiles above), i.e. every block's records reconstructed and laid
out contiguously in HBM.  Inputs are in HBM before timing starts.

Multi-GPU: `--gpus N` runs N ranks, one per GPU -- launched here with torch.distributed.run
when the environment does not already hold them (WORLD_SIZE must equal N otherwise).  Blocks
are independent, so rank r decodes its own 100 k-block shard of one rank-partitioned key space
(synth.cfg2_shard: weak scaling, no data-path collective); the only collectives are the timing
barrier, the max-over-ranks reduction of the time and the sum of the bytes / records decoded.

Prints ONE JSON line on rank 0.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "oxidized-mtbl_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

PIPE_MAX_BLOCK = 49152 - 64  # largest block k_decode_pipe<PipeSmall> stages (decode.hip make_plan)
PIPE_LARGE_MAX_BLOCK = 65664 - 64  # k_decode_pipe<PipeLarge>; bigger -> k_decode_tiles
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E peak, /opt/skills/guides/MI355X_MICROARCH.md (8.0 TB/s spec)


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def host_cores():
    """(CPUs in this process's affinity mask, the cgroup CPU quota in whole CPUs or None)"""
    try:
        ncpu = len(os.sched_getaffinity(0))
    except AttributeError:
        ncpu = os.cpu_count() or 1
    quota = None
    try:   # cgroup v2 "max period" / "quota period"
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            quota = max(1, int(int(q) // int(per)))
    except (OSError, ValueError):
        pass
    return ncpu, quota


def cpu_baseline(data, off, ln, budget_s: float):
    """CPU restatement of src/block.rs (oracle/, reference semantics) on this host's cores:
    one thread per CPU of the affinity mask (fewer only if a cgroup CPU quota caps the process)."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import pyoracle
    pyoracle.build()
    ncpu, quota = host_cores()
    threads = max(1, min(ncpu, quota) if quota else ncpu)
    nblk = off.size
    # 1 thread on a bounded sample, repeated to take >= 1.5 s
    sample = min(nblk, 20_000)
    t1, r1, _ = pyoracle.bench_scan(data, off[:sample], ln[:sample], 1, 1)
    it1 = max(1, int(1.5 / max(t1, 1e-4)))
    t1, r1, _ = pyoracle.bench_scan(data, off[:sample], ln[:sample], 1, it1)
    bytes1 = float(ln[:sample].sum(dtype=np.uint64)) * it1
    # T threads over the whole batch, repeated to fill ~budget_s
    tT, rT, _ = pyoracle.bench_scan(data, off, ln, threads, 1)
    iters = max(1, int(budget_s / max(tT, 1e-3)))
    tT, rT, _ = pyoracle.bench_scan(data, off, ln, threads, iters)
    bytesT = float(ln.sum(dtype=np.uint64)) * iters
    return {
        "value": bytesT / tT / 2**30,
        "unit": "GiB/s",
        "cores": threads,
        "affinity_cpus": ncpu,
        "cgroup_cpu_quota": quota,
        "kind": "port",
        "records_per_s": rT / tT,
        "single_thread_GiBs": bytes1 / t1 / 2**30,
        "single_thread_records_per_s": r1 / t1,
        "sample": f"cfg2 blocks, {threads} threads x {iters} passes over all {nblk} blocks "
                  f"({tT:.1f} s); 1 thread x {it1} passes over the first {sample} blocks ({t1:.2f} s); C restatement of "
                  f"src/block.rs (oracle/mtbl_oracle.c, -O3), reference Rust crate not buildable here",
    }


def pcie_ceiling(nbytes: int = 400 << 20):
    """pinned hipMemcpyAsync rates on this box: H2D alone, D2H alone, both at once (GB/s)"""
    h = torch.empty(nbytes, dtype=torch.uint8).pin_memory()
    h2 = torch.empty(nbytes, dtype=torch.uint8).pin_memory()
    d = torch.empty(nbytes, dtype=torch.uint8, device="cuda")
    d2 = torch.empty(nbytes, dtype=torch.uint8, device="cuda")
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    d.copy_(h, non_blocking=True)
    h2.copy_(d2, non_blocking=True)
    torch.cuda.synchronize()

    def timed(f, reps=4, rounds=3):   # best of `rounds` timings (a ceiling)
        best = 0.0
        for _ in range(rounds):
            t = time.perf_counter()
            for _ in range(reps):
                f()
            torch.cuda.synchronize()
            best = max(best, reps * nbytes / (time.perf_counter() - t) / 1e9)
        return best

    def both():
        with torch.cuda.stream(s1):
            d.copy_(h, non_blocking=True)
        with torch.cuda.stream(s2):
            h2.copy_(d2, non_blocking=True)
    r = {"h2d_GBs": round(timed(lambda: d.copy_(h, non_blocking=True)), 2),
         "d2h_GBs": round(timed(lambda: h2.copy_(d2, non_blocking=True)), 2),
         "bidir_GBs_each": round(timed(both), 2)}
    del h, h2, d, d2
    return r


def end_to_end(data, off, ln, nrec, kbytes, vbytes, reps, dist=None):
    """North-star end-to-end rate: the .mtbl file in (pinned) host memory in, the caller's host
    byte slices out (mtblx_pipe_decode: H2D, decode, D2H on separate streams, 3 chunks in
    flight).  cfg2 as stored (CompressionType::None) and cfg5 = the same records written with
    CompressionType::Snappy (host decompression inside the pipeline, src/compression.rs:116-119).
    Never `value`: reported beside it."""
    from mtblx import codec, pipe, synth
    from mtblx.writer import Writer
    res = {}
    block_bytes = int(ln.sum(dtype=np.uint64))
    res["pcie_ceiling"] = pcie_ceiling()
    pc = res["pcie_ceiling"]
    out = pipe.HostOutputs(off.size, nrec, kbytes, vbytes)
    p = pipe.HostPipe(chunk_bytes=64 << 20, max_blocks=1 << 16, threads=16, device_snappy=False)

    def run(d, o, l, comp, tag, extra=None, pp=None):
        pp = pp or p
        pp.decode(d, o, l, out, compression=comp)    # warm-up (first-touch of pinned pages, slots)
        if dist is not None:
            dist.barrier()
        t0 = time.perf_counter()
        st = None
        h2d = d2h = stage = dec = 0.0
        for _ in range(reps):
            st = pp.decode(d, o, l, out, compression=comp)
            h2d += st.h2d_bytes
            d2h += st.d2h_bytes
            stage += st.stage_seconds
            dec += st.decode_ms
        el = time.perf_counter() - t0
        if dist is not None:
            tt = torch.tensor([el], dtype=torch.float64, device="cuda")
            dist.all_reduce(tt, op=dist.ReduceOp.MAX)
            el = float(tt.item())
        world = dist.get_world_size() if dist is not None else 1
        tot = out.totals
        if int(tot[0]) != nrec or int(tot[1]) != kbytes or int(tot[2]) != vbytes or int(tot[3]) != 0 or \
                not (out.status[: off.size] == 0).all():
            raise RuntimeError(f"end-to-end decode ({tag}) failed: totals={list(tot)}")
        r = {"GiB_per_s": round(block_bytes * reps * world / el / 2**30, 2),
             "records_per_s": round(nrec * reps * world / el, 1),
             "ms_per_pass": round(el * 1e3 / reps, 3), "passes": reps,
             "h2d_GB_per_pass": round(h2d / reps / 1e9, 4), "d2h_GB_per_pass": round(d2h / reps / 1e9, 4),
             "pcie_GBs_h2d": round(h2d / el / 1e9, 2), "pcie_GBs_d2h": round(d2h / el / 1e9, 2),
             "host_stage_ms_per_pass": round(stage * 1e3 / reps, 3),
             "decode_ms_per_pass": round(dec / reps, 3), "chunks": int(st.chunks)}
        # PCIe floor of one pass: each direction's bytes at that direction's best measured
        # rate alone (a true lower bound: a pass cannot move them faster).  The bidirectional
        # figure (both directions at once, the rate measured with both copies in flight) is a
        # model, not a floor -- the pipeline overlaps them only partly -- and reported beside it.
        bound = max(h2d / reps / (pc["h2d_GBs"] * 1e9), d2h / reps / (pc["d2h_GBs"] * 1e9))
        r["pcie_floor_ms_per_pass"] = round(bound * 1e3, 3)
        r["frac_of_pcie_floor"] = round(bound / (el / reps), 3)
        r["bidir_model_ms_per_pass"] = round((h2d + d2h) / reps / (2 * pc["bidir_GBs_each"] * 1e9) * 1e3, 3)
        if extra:
            r.update(extra)
        return r

    pipe.register(data)
    try:
        res["cfg2_none"] = run(data, off, ln, 0, "cfg2")
    finally:
        pipe.unregister(data)
    # cfg5: the cfg2 records written with CompressionType::Snappy (same blocks once decompressed)
    nr_file = int(synth.cfg2_file.last_block_nrec.sum(dtype=np.uint64))
    rk = dist.get_rank() if dist is not None else 0   # the rank's own shard records (synth.cfg2_shard)
    keys, vals, kl, vl = synth.cfg2_arrays(int(off.size * ((4096 - 64) // 79) * 1.02) + 64, seed=synth.SEED_CFG2 + rk,
                                           c0=rk << synth.SHARD_KEY_BITS)
    w = Writer(4096, 16, 1)
    n_in = nr_file
    w.insert_batch(keys[: n_in * kl], np.arange(1, n_in + 1, dtype=np.uint64) * np.uint64(kl), vals[: n_in * vl],
                   np.arange(1, n_in + 1, dtype=np.uint64) * np.uint64(vl))
    zdata = w.into_inner_np()
    zoff, zln = w.block_dir
    zoff, zln = zoff[: off.size].copy(), zln[: off.size].copy()
    # host decompression alone (16 threads), then the device-resident decode of its output
    L = pipe._lib.lib()
    ulen = ln.astype(np.uint64)
    uoff = np.zeros(off.size, np.uint64)
    uoff[1:] = np.cumsum(ulen[:-1], dtype=np.uint64)
    ubuf = np.zeros(int(ulen.sum()), np.uint8)
    zst = np.zeros(off.size, np.int32)
    t0 = time.perf_counter()
    bad = L.mtblx_snappy_decompress_blocks(zdata.ctypes.data, zoff.ctypes.data, zln.ctypes.data, ubuf.ctypes.data,
                                           uoff.ctypes.data, ulen.ctypes.data, zst.ctypes.data, off.size, 16)
    t_dz = time.perf_counter() - t0
    if bad:
        raise RuntimeError("cfg5: host snappy decompression failed")
    batch = codec.DeviceBatch.from_host(ubuf, uoff, ulen.astype(np.uint32))
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        ws = codec.Workspace(batch.nblk)
        dout = codec.DecodedBlocks(batch.nblk, nrec, kbytes, vbytes)
    torch.cuda.synchronize()
    for _ in range(3):
        codec.decode_into(batch, dout, ws, s)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(s)
    for _ in range(20):
        codec.decode_into(batch, dout, ws, s)
    e1.record(s)
    torch.cuda.synchronize()
    dev_ms = e0.elapsed_time(e1) / 20
    if dout.totals_host()[:3] != (nrec, kbytes, vbytes):
        raise RuntimeError("cfg5: device-resident decode of the decompressed blocks failed")
    # f4: device snappy decompression of the same stored blocks (device-resident), then the
    # decode of its output: the same totals
    zb = codec.SnappyBatch.from_host(zdata, zoff, zln)
    lay = codec.SnappyLayout(zb.nblk)
    codec.snappy_dir(zb, lay)
    torch.cuda.synchronize()
    zt = lay.totals.cpu().numpy().view(np.uint64)
    with torch.cuda.stream(s):
        zdst = torch.zeros(int(zt[0]) + 16, dtype=torch.uint8, device="cuda")
        zst_d = torch.zeros(zb.nblk, dtype=torch.int32, device="cuda")
        zdl = torch.zeros(zb.nblk, dtype=torch.int32, device="cuda")
    torch.cuda.synchronize()
    dz = lambda: codec.snappy_decompress_into(zb, lay, zdst, zst_d, zdl, int(zt[1]), s)  # noqa: E731
    for _ in range(3):
        dz()
    dz_ms = _timed(dz, s, 20)
    zbatch = codec.DeviceBatch(zdst, lay.dst_off[: zb.nblk], zdl, int(zt[1]))
    with torch.cuda.stream(s):
        zws = codec.Workspace(zbatch.nblk)
    torch.cuda.synchronize()
    both = lambda: (dz(), codec.decode_into(zbatch, dout, zws, s))  # noqa: E731
    for _ in range(3):
        both()
    both_ms = _timed(both, s, 20)
    if dout.totals_host()[:3] != (nrec, kbytes, vbytes) or int((zst_d != 0).sum().item()) != 0:
        raise RuntimeError("cfg5: device snappy decompression + decode failed")
    pz = pipe.HostPipe(chunk_bytes=64 << 20, max_blocks=1 << 16, threads=16, device_snappy=True)
    pipe.register(zdata)
    try:
        res["cfg5_snappy"] = run(zdata, zoff, zln, 1, "cfg5", {
            "stored_bytes": int(zln.sum(dtype=np.uint64)),
            "host_decompress_GiB_per_s_16_threads": round(block_bytes / t_dz / 2**30, 2),
            "device_resident_GiB_per_s": round(block_bytes / (dev_ms * 1e-3) / 2**30, 1)})
        res["cfg5_snappy_device_decompress"] = run(zdata, zoff, zln, 1, "cfg5-dz", {
            "mode": "MTBLX_PIPE_DEVICE_SNAPPY: stored bytes H2D, mtblx_snappy_decompress_dev + decode on the device",
            "device_resident_decompress_ms": round(dz_ms, 4),
            "device_resident_decompress_GiB_per_s": round(block_bytes / (dz_ms * 1e-3) / 2**30, 1),
            "device_resident_decompress_plus_decode_GiB_per_s": round(block_bytes / (both_ms * 1e-3) / 2**30, 1)},
            pp=pz)
    finally:
        pipe.unregister(zdata)
    res["cfg5_compressible_device"] = compressible_snappy(s)
    res["note"] = ("pinned host file in -> pinned host outputs (keys, values, u32 end offsets, per-block arrays) out; "
                   "PCIe Gen5 x16 (63 GB/s per direction, spec) bounds it; cfg2/cfg5 data are random bytes, so "
                   "snappy stores them nearly uncompressed")
    return res


def compressible_snappy(s, nrec=2_000_000):
    """cfg5 on data snappy actually compresses: cfg1-style records (a 10-digit
    key, the key repeated 1-8 times as the value), written by the product Writer with
    CompressionType::Snappy into 4 KiB blocks (~4.5x), decompressed on the device
    (mtblx_snappy_decompress_dev: its blocks expand > 2x, so k_snappy_lanes takes them) and
    decoded, device-resident.  Checked: every block decompresses, and the
    decode yields every record written."""
    from mtblx import codec, synth
    from mtblx.writer import Writer
    w = Writer(4096, 16, 1)
    n1 = nrec   # ~25 000 blocks of ~80 records
    for k, v in synth.cfg1_records(n1):
        w.insert(k, v)
    z1 = np.frombuffer(w.into_inner(), np.uint8).copy()
    zoff1, zln1 = w.block_dir
    # the file's blocks 4x over (100 000 blocks, the cfg2 / cfg5 batch size; generating 8 M records
    # in Python would take ~40 s): the quad kernel takes 4 blocks per wave, 2048 waves, so 25 000
    # blocks end on a round of 106 busy waves (3.05 rounds -> 4) and read ~13 % low
    rep = 4
    n = n1 * rep
    z = np.tile(z1, rep)
    zoff = np.concatenate([zoff1.astype(np.uint64) + np.uint64(i * z1.size) for i in range(rep)])
    zln = np.tile(zln1, rep)
    zb = codec.SnappyBatch.from_host(z, zoff, zln)
    lay = codec.SnappyLayout(zb.nblk)
    codec.snappy_dir(zb, lay)
    torch.cuda.synchronize()
    zt = lay.totals.cpu().numpy().view(np.uint64)
    with torch.cuda.stream(s):
        dst = torch.zeros(int(zt[0]) + 16, dtype=torch.uint8, device="cuda")
        st = torch.zeros(zb.nblk, dtype=torch.int32, device="cuda")
        dl = torch.zeros(zb.nblk, dtype=torch.int32, device="cuda")
    torch.cuda.synchronize()
    dz = lambda: codec.snappy_decompress_into(zb, lay, dst, st, dl, int(zt[1]), s)  # noqa: E731
    dz()
    torch.cuda.synchronize()
    if int((st != 0).sum().item()) != 0:
        raise RuntimeError("compressible cfg5: device snappy failed")
    out_bytes = int(dl.to(torch.int64).sum().item())
    batch = codec.DeviceBatch(dst, lay.dst_off[: zb.nblk], dl, int(zt[1]))
    with torch.cuda.stream(s):
        ws = codec.Workspace(batch.nblk)
        probe = codec.DecodedBlocks(batch.nblk, 0, 0, 0)
        codec.count_blocks(batch, probe, ws, s)
    s.synchronize()
    nr, kb, vb, _ = probe.totals_host()
    if nr != n:
        raise RuntimeError(f"compressible cfg5: {nr} records decoded, {n} written")
    with torch.cuda.stream(s):
        out = codec.DecodedBlocks(batch.nblk, nr, kb, vb)
    torch.cuda.synchronize()
    _preload(dz, s, 40.0)
    dz_ms = _timed(dz, s, 20)
    both = lambda: (dz(), codec.decode_into(batch, out, ws, s))  # noqa: E731
    both()
    both_ms = _timed(both, s, 20)
    if out.totals_host() != (nr, kb, vb, 0):
        raise RuntimeError("compressible cfg5: decode after device decompression failed")
    stored = int(zln.sum(dtype=np.uint64))
    # end to end (pinned file in -> pinned outputs out, mtblx_pipe_decode) with host and with
    # device decompression: which one MTBLX_PIPE_DEVICE_SNAPPY=auto should pick here
    from mtblx import pipe
    hout = pipe.HostOutputs(int(zb.nblk), nr, kb, vb)
    e2e = {}
    pipe.register(z)
    try:
        for name, mode in (("host_decompress", False), ("device_decompress", True)):
            pp = pipe.HostPipe(chunk_bytes=64 << 20, max_blocks=1 << 16, threads=16, device_snappy=mode)
            pp.decode(z, zoff, zln, hout, compression=1)   # warm-up
            t0 = time.perf_counter()
            for _ in range(3):
                pp.decode(z, zoff, zln, hout, compression=1)
            el = (time.perf_counter() - t0) / 3
            tot = hout.totals
            if int(tot[0]) != nr or int(tot[1]) != kb or int(tot[2]) != vb or int(tot[3]) != 0:
                raise RuntimeError(f"compressible cfg5 end to end ({name}) failed: totals={list(tot)}")
            e2e[name] = {"GiB_per_s_of_block_bytes": round(out_bytes / el / 2**30, 2), "ms_per_pass": round(el * 1e3, 2)}
            del pp
    finally:
        pipe.unregister(z)
    return {"records": n, "blocks": int(zb.nblk), "file_repeats": rep, "stored_bytes": stored, "decompressed_bytes": out_bytes,
            "end_to_end": e2e,
            "ratio": round(out_bytes / stored, 2),
            "kernel": "k_snappy_lanes (blocks expanding > 2x; MTBLX_SNAPPY_KERNEL=" + os.environ.get("MTBLX_SNAPPY_KERNEL", "auto") + ")",
            "device_decompress_ms": round(dz_ms, 4),
            "device_decompress_GB_per_s_out": round(out_bytes / (dz_ms * 1e-3) / 1e9, 1),
            "device_decompress_plus_decode_GiB_per_s": round(out_bytes / (both_ms * 1e-3) / 2**30, 1)}


_PRELOAD_TRACE = []
_T_PRE_END = 0.0


def _preload(step, stream, ms):
    """Untimed: run `step` back to back until ~`ms` of GPU time has passed.  The MI355X drops
    its clocks after ~0.5 s idle and needs ~15 ms of this load to ramp back (the first ~80
    cfg2 launches after idle run 0.178 -> 0.190 -> ... -> 0.1546 ms: scripts/warm_probe.py,
    profiles/r02/final/warm.log); other kernels (the copy sweep, the CRC) do not hold the
    clock for it.  Runs right before the W warmup steps, outside the timed region."""
    if ms <= 0:
        return 0
    n, t0 = 0, time.perf_counter()
    while True:
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        with torch.cuda.stream(stream):
            e0.record(stream)
            for _ in range(10):
                step()
            e1.record(stream)
        e1.synchronize()
        n += 10
        dt = e0.elapsed_time(e1)
        ms -= dt
        if os.environ.get("MTBLX_BENCH_CHUNKS"):
            _PRELOAD_TRACE.append(round(dt / 10, 4))
        if ms <= 0 or time.perf_counter() - t0 > 5.0:
            return n


def _timed(fn, stream, reps):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    for _ in range(reps):
        fn()
    e1.record(stream)
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


def _reduce_over_ranks(x, dist, op: str, device="cuda"):
    if dist is None:
        return x
    t = torch.tensor([x], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX if op == "max" else dist.ReduceOp.SUM)
    return float(t.item())


def _max_over_ranks(x, dist, device="cuda"):
    return _reduce_over_ranks(x, dist, "max", device)


def _sum_over_ranks(x, dist, device="cuda"):
    return _reduce_over_ranks(x, dist, "sum", device)


def launch_command(args_list, gpus: int, port: int):
    """the torch.distributed.run command that runs this script as `gpus` ranks"""
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={gpus}",
            "--master-addr", "127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + list(args_list)


def maybe_launch(args, argv) -> int | None:
    """--gpus N > 1 outside torchrun: start the N ranks as a child process (before this process
    touches the GPU: torch.cuda.device_count() does not initialise it) and return its exit code;
    None when this process is a rank (or N == 1) and goes on."""
    if args.gpus <= 1 or "WORLD_SIZE" in os.environ:
        return None
    nvis = torch.cuda.device_count()
    if nvis < args.gpus and not args.share_gpu:
        log(f"--gpus {args.gpus}: only {nvis} GPU(s) visible")
        return 2
    import socket
    sk = socket.socket()
    sk.bind(("127.0.0.1", 0))
    port = sk.getsockname()[1]
    sk.close()
    import subprocess
    return subprocess.call(launch_command(argv, args.gpus, port))


def init_ranks(args, backend: str = "nccl"):
    """rank set-up from the torchrun environment -> (dist or None, world, rank, local).  The
    world must be the --gpus the run was asked for."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"WORLD_SIZE={world} but --gpus {args.gpus}: launch with --nproc-per-node {args.gpus}")
    if backend == "nccl":
        if torch.cuda.device_count() < world:
            raise SystemExit(f"--gpus {world}: only {torch.cuda.device_count()} GPU(s) visible")
        torch.cuda.set_device(local)
    elif getattr(args, "share_gpu", False):
        torch.cuda.set_device(0)
    dist = None
    if world > 1:
        import torch.distributed as dist
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
    return dist, world, rank, local


def rank_totals(block_bytes: int, nrec: int, elapsed: float, dist, device="cuda"):
    """whole-job totals: (bytes over all ranks, records over all ranks, max elapsed)"""
    return (int(_sum_over_ranks(float(block_bytes), dist, device)), int(_sum_over_ranks(float(nrec), dist, device)),
            _max_over_ranks(elapsed, dist, device))


def get_leg(data, nblocks, rank, nq=1 << 20, reps=10):
    """f2, Reader::get batched on the device (mtblx_get, src/reader.rs:111-122): nq queries on the
    bench's cfg2 file, half of them keys the file holds (random records), half absent (a present
    key with one tail byte changed: its counter prefix is unique, so the key is not in the file),
    keys already in HBM; checksums on (the reference default: every landed block's CRC) and off.
    Device time per batch by HIP events; every found value must be the record's 64 bytes."""
    import ctypes as C
    from mtblx import _lib as mlib, codec, reader, synth
    nrec = synth.cfg2_file_nrec(nblocks)
    keys = synth.cfg2_keys(nrec, seed=synth.SEED_CFG2 + rank, c0=rank << synth.SHARD_KEY_BITS)
    rng = np.random.default_rng(0x6765740)
    q = keys[rng.integers(0, nrec, nq)].copy()
    q[nq // 2:, 15] ^= 0x5A
    r = reader.Reader(data, verify_checksums=True)
    dev = r.file.device
    kb = torch.from_numpy(q.reshape(-1)).to(dev)
    ke = torch.arange(1, nq + 1, dtype=torch.int64, device=dev) * 16
    st = torch.empty(nq, dtype=torch.int32, device=dev)
    vo = torch.empty(nq, dtype=torch.int64, device=dev)
    vl = torch.empty(nq, dtype=torch.int64, device=dev)
    s = torch.cuda.Stream()
    L = mlib.lib()
    out = {"queries": nq, "present": nq // 2}
    for verify in (1, 0):
        def call():
            if L.mtblx_get(C.c_void_p(r.file.data_ptr()), r.len, r.version, verify, r.index_off, r.index_len,
                           C.c_void_p(kb.data_ptr()), C.c_void_p(ke.data_ptr()), nq, C.c_void_p(st.data_ptr()),
                           C.c_void_p(vo.data_ptr()), C.c_void_p(vl.data_ptr()), C.c_void_p(s.cuda_stream)) != 0:
                raise RuntimeError("mtblx_get failed")
        with torch.cuda.stream(s):
            call()
            call()
            ms = _timed(call, s, reps)
        torch.cuda.synchronize()
        found = int((st == mlib.GET_FOUND).sum().item())
        ok = found == nq // 2 and bool((vl[st == mlib.GET_FOUND] == 64).all().item())
        out["checksums_on" if verify else "checksums_off"] = {
            "ms": round(ms, 3), "gets_per_s": round(nq / (ms * 1e-3), 1), "found": found, "checked": ok}
    del r
    return out


def run_cfg3(args, dist, world, rank):
    """BASELINE configs[2]: 1 M blocks x 64 KiB per GPU, Zipf 8..256 B keys, 64 B values,
    restart interval 16 -- device encode (Writer block cut + BlockBuilder + framing, src/writer.rs,
    src/block_builder.rs) and decode round trip, bit-exact (every record compared on the device).
    Generated and processed in chunks of `--cfg3-chunk` blocks (HBM holds records, blocks and
    decoded outputs of one chunk at a time); kernel times are summed over chunks."""
    from mtblx import codec, encode, synth
    s = torch.cuda.Stream()
    total_blocks = args.cfg3_blocks
    per_chunk = args.cfg3_chunk
    rec_per_blk = 640   # ~637 records per 64 KiB block at this key/value mix
    c0 = 0
    acc = dict(blocks=0, records=0, block_bytes=0, key_bytes=0, val_bytes=0, enc_ms=0.0, dec_ms=0.0, plan_ms=0.0,
               file_bytes=0, mismatches=0, chunks=0)
    done = 0
    ci = 0
    # the block cut's scratch (caller-owned, mtblx_plan_workspace_bytes), sized once for the largest chunk
    pws = encode.PlanWorkspace(int(min(per_chunk, total_blocks) * rec_per_blk * 1.03) + 1024, 64, 16, keep=True)
    while done < total_blocks:
        want = min(per_chunk, total_blocks - done)
        nrec = int(want * rec_per_blk * 1.03) + 1024
        recs, c_last = synth.cfg3_records_device(nrec, seed=synth.SEED_CFG3 + 1000 * rank + ci, c0=c0)
        c0 = c_last
        nsh = 64
        cuts = torch.linspace(0, nrec, nsh + 1, device="cuda").to(torch.int64)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        # the Writer's block cut, its sums kept for the encode (mtblx_encode_plan_keep)
        blk, kept = encode.plan(recs, 65536, 16, shard_rec=cuts, keep=True, workspace=pws)
        acc["plan_ms"] += (time.perf_counter() - t0) * 1e3
        blk = blk[: want + 1].contiguous()
        nb = int(blk.numel()) - 1
        bufs = encode.EncodeBuffers(recs, nb)
        with torch.cuda.stream(s):
            # reference: the self-contained encode (size pass + look-back), then the product
            # planned encode (mtblx_encode_blocks_planned) whose output the round trip checks
            encode.encode_into(recs, blk, bufs, 16, True, s)
            acc["enc_unplanned_ms"] = acc.get("enc_unplanned_ms", 0.0) + _timed(
                lambda: encode.encode_into(recs, blk, bufs, 16, True, s), s, 3)
            encode.encode_into(recs, blk, bufs, 16, True, s, plan=kept)      # warm-up
            enc_ms = _timed(lambda: encode.encode_into(recs, blk, bufs, 16, True, s, plan=kept), s, 3)
        if os.environ.get("MTBLX_ENC_STAMPS_PRINT") and ci == 0:   # diagnostic build (make variant_enc, -DMTBLX_ENC_STAMPS)
            torch.cuda.synchronize()
            d = bufs.ws[:128].cpu().numpy().view(np.uint64).astype(np.float64)
            names = ["tables+ticket", "phaseA", "assemble", "lookback", "crc", "stream"]
            log("[enc stamps] cycles per block (thread 0, after a barrier): " + json.dumps(
                {n: round(d[2 + k] / max(d[15], 1), 1) for k, n in enumerate(names)}))
        e = encode.Encoded(bufs.out, bufs.blk_off[:nb], bufs.blk_len[:nb], bufs.status[:nb], bufs.totals)
        if int(e.totals[1].item()) != 0:
            raise RuntimeError("cfg3: encode reported a failed block")
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
            dec_ms = _timed(lambda: codec.decode_into(batch, out, ws, s), s, 5)
        if args.stamps and ci == 0:   # diagnostic build: per-phase cycles per tile of this chunk's decode
            torch.cuda.synchronize()
            d = ws.buf[:128].cpu().numpy().view(np.uint64).astype(np.float64)
            names = ["copy:wait-ready", "w1:lookback+barrier", "w0:walk-loop", "w0:scan-publish",
                     "loader:dma-issue", "copy:barrier", "loader:dma-wait", "copy:copy", "w0:barrier",
                     "w0:trailers", "w0:interval-setup", "w1:barrier", "loader:barrier",
                     "copy:barrier-min-over-waves", "copy:prepare-max-over-waves"]
            acc["phase_cycles_per_tile"] = {n: round(d[k] / max(d[15], 1), 1) for k, n in enumerate(names)}
        # round trip: every decoded record == the generated record
        r_used = int(blk[-1].item())
        ke_used = int(recs.key_end[r_used - 1].item())
        ok = nr == r_used and kb == ke_used and vb == 64 * r_used and out.totals_host()[3] == 0
        ok = ok and bool((out.status[:nb] == 0).all().item())
        ok = ok and torch.equal(out.keys[:kb], recs.keys[:kb]) and torch.equal(out.vals[:vb], recs.vals[:vb])
        if ok:
            nrb = out.nrec[:nb].to(torch.int64)
            blk_of = torch.repeat_interleave(torch.arange(nb, device="cuda"), nrb)
            ke = out.key_base[:nb][blk_of] + (out.key_end[:nr].to(torch.int64) & 0xFFFFFFFF)
            ok = torch.equal(ke, recs.key_end[:nr])
        acc["mismatches"] += 0 if ok else 1
        acc["blocks"] += nb
        acc["records"] += nr
        acc["block_bytes"] += int(e.blk_len.to(torch.int64).sum().item())
        acc["file_bytes"] += int(e.totals[0].item())
        acc["key_bytes"] += kb
        acc["val_bytes"] += vb
        acc["enc_ms"] += enc_ms
        acc["dec_ms"] += dec_ms
        acc["chunks"] += 1
        done += nb
        ci += 1
        log(f"[rank {rank}] cfg3 chunk {ci}: {nb} blocks, enc {enc_ms:.2f} ms, dec {dec_ms:.2f} ms, ok={ok}")
        del recs, blk, bufs, e, batch, ws, probe, out, kept
        torch.cuda.empty_cache()
    if acc["mismatches"]:
        raise RuntimeError(f"cfg3 round trip failed in {acc['mismatches']} chunk(s)")
    dec_ms = _max_over_ranks(acc["dec_ms"], dist)
    enc_ms = _max_over_ranks(acc["enc_ms"], dist)
    bb = acc["block_bytes"] * world
    alg_dec = acc["block_bytes"] + acc["key_bytes"] + acc["val_bytes"] + 8 * acc["records"] + 24 * acc["blocks"]
    alg_enc = acc["key_bytes"] + acc["val_bytes"] + 16 * acc["records"] + acc["file_bytes"] + 8 * acc["blocks"]
    return {
        "metric": "cfg3 round trip: GiB/s of block bytes decoded / encoded, device-resident",
        "value": round(bb / (dec_ms * 1e-3) / 2**30, 2), "unit": "GiB/s", "n_gpus": world,
        "decode_records_per_s": round(acc["records"] * world / (dec_ms * 1e-3), 1),
        "encode_GiB_per_s": round(bb / (enc_ms * 1e-3) / 2**30, 2),
        "encode_unplanned_GiB_per_s": round(bb / (_max_over_ranks(acc.get("enc_unplanned_ms", 0.0), dist) * 1e-3) / 2**30, 2),
        "encode_records_per_s": round(acc["records"] * world / (enc_ms * 1e-3), 1),
        "plan_ms_total": round(acc["plan_ms"], 1),
        # the device Writer end to end: block cut (mtblx_encode_plan, wall clock per chunk) + encode
        "writer_GiB_per_s": round(bb / ((enc_ms + _max_over_ranks(acc["plan_ms"], dist)) * 1e-3) / 2**30, 2), "scaling": "weak", "dtype": "u8",
        "data": "synthetic (device generator: Zipf 8..256 B keys = be64(counter) || random tail, 64 B random values)",
        "config": {"workload": "cfg3: 64 KiB blocks, restart_interval=16, compression=none, encode (framed) + decode",
                   "blocks_per_gpu": acc["blocks"], "records_per_gpu": acc["records"],
                   "block_bytes_per_gpu": acc["block_bytes"], "chunks": acc["chunks"]},
        "round_trip": "bit-exact (keys, values, key END offsets of every record; all statuses OK)",
        **({"phase_cycles_per_tile": acc["phase_cycles_per_tile"]} if "phase_cycles_per_tile" in acc else {}),
        "roofline": {"decode": {"kernel": "k_decode_pipe<PipeLarge>", "achieved_GBs":
                                round(alg_dec / (acc["dec_ms"] * 1e-3) / 1e9, 1), "peak": HBM_PEAK_GBS,
                                "alg_bytes": alg_dec},
                     "encode": {"kernel": "k_encode<true> (planned)", "achieved_GBs": round(alg_enc / (acc["enc_ms"] * 1e-3) / 1e9, 1),
                                "peak": HBM_PEAK_GBS, "alg_bytes": alg_enc}},
    }


def run_cfg4(args, dist, world, rank):
    """BASELINE configs[3]: 10 GiB of blocks in equal byte thirds of 4, 16 and 64 KiB blocks
    (three .mtbl files, cfg2 key/value scheme) = ONE global block directory, cut into `world`
    byte-balanced contiguous shards by mtblx.shard.shard_cuts (the product sharding, no
    collective).  Every rank builds the same files (same seeds; written on the device by the
    encode path, byte-identical to the Writer: tests/test_encode_gpu.py), takes its cut, and
    decodes it per file piece (a piece = its cut intersected with one file, one
    mtblx_decode_blocks call each).  Device-resident decode per step, then the end-to-end pipe
    (pinned host file in, pinned host outputs out) over the same pieces."""
    from mtblx import codec, encode, pipe, shard
    s = torch.cuda.Stream()
    per_leg = int(args.cfg4_gib * 2**30 / 3)
    files = []
    for li, bs in enumerate((4096, 16384, 65536)):
        nrec = per_leg // 83 + 1024     # ~80 B of payload + header per record
        g = torch.Generator(device="cuda")
        g.manual_seed(0x6D74626C04 + li)          # the same files on every rank
        gaps = torch.randint(1, 1 << 20, (nrec,), generator=g, device="cuda", dtype=torch.int64)
        c = torch.cumsum(gaps, 0)
        keys = torch.randint(0, 256, (nrec, 16), generator=g, device="cuda", dtype=torch.uint8)
        for j in range(8):
            keys[:, j] = ((c >> (8 * (7 - j))) & 0xFF).to(torch.uint8)
        vals = torch.randint(0, 256, (nrec * 64,), generator=g, device="cuda", dtype=torch.uint8)
        recs = encode.DeviceRecords(keys.reshape(-1), torch.arange(1, nrec + 1, device="cuda") * 16, vals,
                                    torch.arange(1, nrec + 1, device="cuda") * 64)
        blk = encode.plan(recs, bs, 16)
        e = encode.encode_blocks(recs, blk, 16, framed=True).check()
        ends = torch.cumsum(e.blk_len.to(torch.int64), 0)
        nb = int((ends <= per_leg).sum().item())     # the leg's byte budget, whole blocks
        file_len = int(e.blk_off[nb - 1].item()) + int(e.blk_len[nb - 1].item())
        files.append(dict(bs=bs, nb=nb, data=e.out[:file_len].clone(), off=e.blk_off[:nb].clone(),
                          ln=e.blk_len[:nb].clone(), blk_rec=blk[: nb + 1].clone()))
        del recs, keys, vals, gaps, c, blk, e
        torch.cuda.empty_cache()
    # one global directory (file 0's blocks, then file 1's, then file 2's) -> this rank's cut
    gl = np.concatenate([f["ln"].cpu().numpy().view(np.uint32) for f in files])
    cuts = shard.shard_cuts(gl, world)
    c0, c1 = int(cuts[rank]), int(cuts[rank + 1])
    pieces, base = [], 0
    for f in files:
        lo, hi = max(c0 - base, 0), min(c1 - base, f["nb"])
        if lo < hi:
            off, ln = f["off"][lo:hi], f["ln"][lo:hi]
            nr = int((f["blk_rec"][hi] - f["blk_rec"][lo]).item())
            batch = codec.DeviceBatch(f["data"], off, ln, int(ln.max().item()))
            with torch.cuda.stream(s):
                ws = codec.Workspace(hi - lo)
                out = codec.DecodedBlocks(hi - lo, nr, 16 * nr, 64 * nr)
            pieces.append(dict(bs=f["bs"], lo=lo, hi=hi, nb=hi - lo, nr=nr, bytes=int(ln.to(torch.int64).sum().item()),
                               batch=batch, ws=ws, out=out, file=f))
        base += f["nb"]
    torch.cuda.synchronize()

    def step():
        for P in pieces:
            codec.decode_into(P["batch"], P["out"], P["ws"], s)
    _preload(step, s, args.preload_ms)
    with torch.cuda.stream(s):
        for _ in range(args.warmup):
            step()
    torch.cuda.synchronize()
    for P in pieces:
        h = P["out"].totals_host()
        if h != (P["nr"], 16 * P["nr"], 64 * P["nr"], 0) or not bool((P["out"].status[: P["nb"]] == 0).all().item()):
            raise RuntimeError(f"cfg4 piece {P['bs']}: decode mismatch {h}")
    # per leg: its own preload first.  The host checks above leave the GPU idle for ~40 ms, and
    # the first ~30 back-to-back launches after an idle period run up to 35 % slow while the
    # clocks settle (profiles/r03/a: cfg2 at this leg's size goes 1.25 -> 1.65 -> 1.20 ms); timing
    # 10 launches straight after the checks measured that transient, not the leg
    per_leg_ms = {}
    with torch.cuda.stream(s):
        for P in pieces:
            leg = lambda P=P: codec.decode_into(P["batch"], P["out"], P["ws"], s)  # noqa: E731
            _preload(leg, s, args.preload_ms)
            per_leg_ms[P["bs"]] = _timed(leg, s, 20)
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    with torch.cuda.stream(s):
        for _ in range(args.steps):
            step()
    torch.cuda.synchronize()
    el = _max_over_ranks(time.perf_counter() - t0, dist)
    my_bytes = sum(P["bytes"] for P in pieces)
    my_recs = sum(P["nr"] for P in pieces)
    tot_bytes = int(gl.astype(np.uint64).sum())
    tot_recs = sum(int(f["blk_rec"][-1].item()) for f in files)
    res = {"metric": "cfg4: GiB/s of block bytes decoded, device-resident (mixed 4/16/64 KiB)",
           "value": round(tot_bytes / (el / args.steps) / 2**30, 2), "unit": "GiB/s", "n_gpus": world,
           "records_per_s": round(tot_recs / (el / args.steps), 1), "steps": args.steps,
           "ms_per_step": round(el * 1e3 / args.steps, 3),
           "scaling": "strong (one 10 GiB directory cut into n_gpus byte-balanced shards)",
           "dtype": "u8", "data": "synthetic cfg2 scheme, written on the device by the encode path",
           "config": {"workload": "cfg4: 10 GiB total, equal byte thirds of 4/16/64 KiB blocks, one directory "
                                  "sharded by mtblx.shard.shard_cuts",
                      "total_GiB": args.cfg4_gib, "total_bytes": tot_bytes, "total_records": tot_recs,
                      "rank0_cut_blocks": [c0, c1], "rank0_bytes": my_bytes, "rank0_records": my_recs},
           "legs": {str(P["bs"]): {"blocks": P["nb"], "bytes": P["bytes"], "decode_ms": round(per_leg_ms[P["bs"]], 3),
                                   "GiB_per_s": round(P["bytes"] / (per_leg_ms[P["bs"]] * 1e-3) / 2**30, 1)}
                    for P in pieces}}
    # end-to-end per piece: pinned host file in, pinned host outputs out
    if not args.no_e2e:
        for P in pieces:
            del P["batch"], P["ws"], P["out"]
        torch.cuda.empty_cache()
        p = pipe.HostPipe(chunk_bytes=64 << 20, threads=16)
        hosts = []
        for P in pieces:
            hosts.append((P, P["file"]["data"].cpu().numpy(), P["file"]["off"][P["lo"]:P["hi"]].cpu().numpy().astype(np.uint64),
                          P["file"]["ln"][P["lo"]:P["hi"]].cpu().numpy().view(np.uint32).copy()))
        outs = [pipe.HostOutputs(P["nb"], P["nr"], 16 * P["nr"], 64 * P["nr"]) for P in pieces]
        for (P, hd, ho, hl), o in zip(hosts, outs):
            pipe.register(hd)
            p.decode(hd, ho, hl, o)      # warm-up: pinned pages, slot buffers
        if dist is not None:
            dist.barrier()
        t0 = time.perf_counter()
        legs_e2e = {}
        for (P, hd, ho, hl), o in zip(hosts, outs):
            t1 = time.perf_counter()
            p.decode(hd, ho, hl, o)
            legs_e2e[str(P["bs"])] = time.perf_counter() - t1
        dt = _max_over_ranks(time.perf_counter() - t0, dist)
        for (P, hd, ho, hl), o in zip(hosts, outs):
            pipe.unregister(hd)
            if tuple(int(x) for x in o.totals) != (P["nr"], 16 * P["nr"], 64 * P["nr"], 0):
                raise RuntimeError("cfg4 end-to-end decode mismatch")
            res["legs"][str(P["bs"])]["end_to_end_GiB_per_s"] = round(P["bytes"] / legs_e2e[str(P["bs"])] / 2**30, 2)
        res["end_to_end_GiB_per_s"] = round(tot_bytes / dt / 2**30, 2)
    return res


def parse_args(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--share-gpu", action="store_true",
                    help="diagnostic: the --gpus N ranks all on GPU 0 with gloo collectives -- exercises the "
                         "multi-rank path (launch, shards, barriers, max-over-ranks) on a 1-GPU box; not scaling")
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--blocks", type=int, default=100_000)
    ap.add_argument("--block-size", type=int, default=4096,
                    help="diagnostic: writer block size (cfg2 = 4096; cfg4 also uses 16384 / 65536)")
    ap.add_argument("--cpu-seconds", type=float, default=8.0)
    ap.add_argument("--preload-ms", type=float, default=40.0,
                    help="untimed decode launches before the W warmup steps, to bring the GPU clocks to their "
                         "loaded state (0 = off)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-ceiling", action="store_true", help="skip the stream-copy ceiling measurement")
    ap.add_argument("--no-crc", action="store_true", help="skip the CRC-32C verify measurement")
    ap.add_argument("--no-e2e", action="store_true", help="skip the end-to-end (host in, host out) measurement")
    ap.add_argument("--no-get", action="store_true", help="skip the batched Reader::get leg (f2)")
    ap.add_argument("--e2e-passes", type=int, default=5)
    ap.add_argument("--config", default="cfg2", choices=["cfg2", "cfg3", "cfg4"],
                    help="cfg2 (default, BASELINE configs[1]: the metric's workload); cfg3 / cfg4 print their own line")
    ap.add_argument("--cfg3-blocks", type=int, default=1_000_000)
    ap.add_argument("--cfg3-chunk", type=int, default=100_000)
    ap.add_argument("--cfg4-gib", type=float, default=10.0)
    ap.add_argument("--lib", default=None, help="diagnostic: alternative libmtblx build (ablations)")
    ap.add_argument("--stamps", action="store_true",
                    help="diagnostic: load libmtblx_stamps.so and report per-phase cycles per tile (not a measurement)")
    ap.add_argument("--traffic-json", default=os.path.join(ROOT, "profiles", "traffic.json"),
                    help="PMC-derived HBM bytes per decode launch (profiles/, written by scripts/pmc_traffic.py "
                         "from rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes)")
    return ap.parse_args(argv)


def main():
    argv = sys.argv[1:]
    args = parse_args(argv)
    rc = maybe_launch(args, argv)
    if rc is not None:
        sys.exit(rc)

    if args.stamps or (args.lib and not os.environ.get("MTBLX_AB_CRC")):
        args.no_crc = True    # diagnostic builds: decode timing only (MTBLX_AB_CRC=1: keep the CRC legs)
    if args.stamps:
        os.environ["MTBLX_LIB"] = args.lib or os.path.join(ROOT, "oxidized-mtbl_amd", "mtblx", "libmtblx_stamps.so")
    elif args.lib:
        os.environ["MTBLX_LIB"] = args.lib
    dist, world, rank, local = init_ranks(args, backend="gloo" if args.share_gpu else "nccl")
    if args.share_gpu and world > 1:   # each rank's look-back launches stay co-resident on its CUs
        os.environ["MTBLX_PIPE_CUS"] = str(max(1, torch.cuda.get_device_properties(0).multi_processor_count // world))

    from mtblx import codec, synth

    if args.config in ("cfg3", "cfg4"):
        res = (run_cfg3 if args.config == "cfg3" else run_cfg4)(args, dist, world, rank)
        if rank == 0:
            print(json.dumps(res), flush=True)
        if dist is not None:
            dist.destroy_process_group()
        return

    t = time.time()
    data, off, ln = synth.cfg2_shard(rank, world, args.blocks, block_size=args.block_size)
    exp_nrec = int(synth.cfg2_file.last_block_nrec.sum(dtype=np.uint64))  # records the Writer put in these blocks
    log(f"[rank {rank}] generated {off.size} blocks / {data.size / 2**20:.1f} MiB in {time.time() - t:.1f}s")
    batch = codec.DeviceBatch.from_host(data, off, ln)
    stream = torch.cuda.Stream()
    # every buffer is allocated (and zero-filled) on `stream`, the stream the decode runs on
    with torch.cuda.stream(stream):
        ws = codec.Workspace(batch.nblk)
        probe = codec.DecodedBlocks(batch.nblk, 0, 0, 0)
        codec.count_blocks(batch, probe, ws, stream)
    stream.synchronize()
    nrec, kbytes, vbytes, _ = probe.totals_host()
    with torch.cuda.stream(stream):
        out = codec.DecodedBlocks(batch.nblk, nrec, kbytes, vbytes)
    torch.cuda.synchronize()
    del probe
    block_bytes = int(ln.sum(dtype=np.uint64))

    # algorithmic bytes per decode launch: block bytes read +
    # key/value bytes written + 2 x u32 end offsets per record + 24 B of per-block outputs
    alg_bytes = block_bytes + kbytes + vbytes + 8 * nrec + 24 * batch.nblk

    # stream-copy ceiling on this box, measured before the decode steps: the in-repo gfx950 copy kernel
    #     (mtblx_stream_copy: 16 B per lane, 1-8 accesses in flight, optional non-temporal
    #     stores / loads) moving the same number of bytes (half read, half written) as one
    #     decode launch; best variant of the sweep
    ceiling, ceiling_variant = None, None
    if not args.no_ceiling:
        from mtblx import _lib as mlib
        CL = mlib.lib()
        half = (alg_bytes // 2) & ~15
        with torch.cuda.stream(stream):
            src = torch.empty(half, dtype=torch.uint8, device="cuda")
            dst = torch.empty(half, dtype=torch.uint8, device="cuda")
            src.fill_(1)
        torch.cuda.synchronize()
        hs = int(stream.cuda_stream)
        # two rounds of 20 timed copies per variant (~50 ms of GPU work: a steadier best-of, and
        # the clocks are at their loaded state when the decode steps start)
        for _round in range(2):
            for var in (1, 2, 3, 2 | 4, 3 | 4, 2 | 12, 3 | 12):
                def cp(v=var):
                    if CL.mtblx_stream_copy(dst.data_ptr(), src.data_ptr(), half, v, hs) != 0:
                        raise RuntimeError("mtblx_stream_copy failed")
                for _ in range(2):
                    cp()
                c_ms = _timed(cp, stream, 20)
                gbs = 2 * half / (c_ms * 1e-3) / 1e9
                if ceiling is None or gbs > ceiling:
                    ceiling, ceiling_variant = gbs, var
        del src, dst
        torch.cuda.empty_cache()

    # The f1 legs (CRC-32C verify, decode + verify) run here, BEFORE the decode's warmup and
    # timed steps: they decode the same batch into the same buffers, so the timed steps start
    # with the GPU at its loaded state (a 20-step run after only the copy-ceiling sweep read
    # ~7 % slower per launch than a 200-step one: profiles/r02/final).  Nothing in the timed
    # region changes: W warmup steps, then exactly K timed decode launches.
    # f1: device CRC-32C verify of the same blocks (separate kernel; the stored checksums sit
    # right before each content in the file the batch addresses)
    crc_info = None
    if not args.no_crc:
        with torch.cuda.stream(stream):
            crc, bad = codec.crc32c_blocks(batch, framed=True, stream=stream)
        torch.cuda.synchronize()
        _preload(lambda: codec.crc32c_blocks(batch, framed=True, stream=stream), stream, args.preload_ms)
        with torch.cuda.stream(stream):
            c0, c1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            c0.record(stream)
            for _ in range(10):
                codec.crc32c_blocks(batch, framed=True, stream=stream)
            c1.record(stream)
        torch.cuda.synchronize()
        crc_ms = c0.elapsed_time(c1) / 10
        # f1 fused: decode + checksum in one launch (the Reader's default verify_checksums path)
        vbad = torch.zeros(batch.nblk, dtype=torch.uint8, device="cuda")
        with torch.cuda.stream(stream):
            for _ in range(3):
                codec.decode_verify_into(batch, out, ws, None, vbad, True, stream, fused=True)
            v_ms = _timed(lambda: codec.decode_verify_into(batch, out, ws, None, vbad, True, stream, fused=True),
                          stream, 20)
        hv = out.totals_host()
        if hv != (nrec, kbytes, vbytes, 0) or int(vbad.sum().item()) != 0:
            raise RuntimeError(f"fused verify decode mismatch: {hv}")
        # the default mtblx_decode_blocks_verify: the decode, then the CRC kernel, one stream
        vbad.zero_()
        torch.cuda.synchronize()
        _preload(lambda: codec.decode_verify_into(batch, out, ws, None, vbad, True, stream, fused=False), stream,
                 args.preload_ms)
        with torch.cuda.stream(stream):
            for _ in range(3):
                codec.decode_verify_into(batch, out, ws, None, vbad, True, stream, fused=False)
            d_ms = _timed(lambda: codec.decode_verify_into(batch, out, ws, None, vbad, True, stream, fused=False),
                          stream, 20)
        hv = out.totals_host()
        if hv != (nrec, kbytes, vbytes, 0) or int(vbad.sum().item()) != 0:
            raise RuntimeError(f"decode+verify mismatch: {hv}")
        ck = "k_crc32c_blocks" if os.environ.get("MTBLX_CRC_KERNEL", "").startswith("l") else "k_crc32c_mfma"
        crc_info = {"kernel": ck, "ms": round(crc_ms, 4),
                    "GiB_per_s": round(block_bytes / (crc_ms * 1e-3) / 2**30, 1),
                    "bad_blocks": int(bad.sum().item()),
                    "decode_blocks_verify": {"kernels": "k_decode_pipe<PipeSmall> + " + ck, "ms": round(d_ms, 4),
                                             "GiB_per_s": round(block_bytes / (d_ms * 1e-3) / 2**30, 1)},
                    "fused_decode_verify": {"kernel": "k_decode_pipe<PipeSmallV>", "ms": round(v_ms, 4),
                                            "GiB_per_s": round(block_bytes / (v_ms * 1e-3) / 2**30, 1),
                                            "vs_decode_then_crc_GiB_per_s": None}}

    def step():
        # one mtblx_decode_blocks call = one decode kernel launch (no fills: the workspace resets itself)
        codec.decode_into(batch, out, ws, stream)

    # validity first (one launch, then host checks whose first use loads torch kernels: ~90 ms
    # of host time with the GPU idle, long enough for it to drop its clocks), and the first
    # barrier (communicator set-up) -- both before the preload, so that preload -> W warmup
    # steps -> timed steps run back to back
    with torch.cuda.stream(stream):
        step()
    torch.cuda.synchronize()
    h = out.totals_host()
    st = out.status[: batch.nblk]
    # validity: every block OK and the decoded totals equal what the Writer wrote (16 B keys, 64 B values)
    if h[3] != 0 or not bool((st == 0).all().item()) or h[0] != exp_nrec or h[1] != 16 * exp_nrec \
            or h[2] != 64 * exp_nrec:
        if args.lib:
            log(f"(ablation build) totals={h}")
        else:
            raise RuntimeError(f"decode failed: totals={h}, bad blocks={int((st != 0).sum().item())}")
    if dist is not None:
        dist.barrier()
    n_pre = _preload(step, stream, args.preload_ms)
    global _T_PRE_END
    _T_PRE_END = time.perf_counter()
    with torch.cuda.stream(stream):
        for _ in range(args.warmup):
            step()
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize()
    # HIP events on the decode stream bracket the timed region (one pair: an event between two
    # launches costs ~10 us of idle GPU per step on this stack); the launches run back to back,
    # so region / K is the kernel's average launch duration (rocprofv3 agrees: profiles/)
    e_start, e_end = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    with torch.cuda.stream(stream):
        e_start.record(stream)
        for i in range(args.steps):
            step()
        e_end.record(stream)
    t_enq = time.perf_counter() - t0   # host time to enqueue the K steps (must stay below the GPU time)
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    if dist is not None:
        dist.barrier()
    block_bytes = int(ln.sum(dtype=np.uint64))
    total_bytes, total_recs, elapsed = rank_totals(block_bytes, int(nrec), elapsed, dist)

    k_decode_ms = e_start.elapsed_time(e_end) / args.steps
    if out.totals_host() != h:   # the timed launches decoded the same totals
        raise RuntimeError(f"decode totals changed over the timed steps: {out.totals_host()} vs {h}")
    if os.environ.get("MTBLX_BENCH_CHUNKS"):   # diagnostic: per-chunk launch time after the timed region
        cs = []
        for _ in range(int(os.environ["MTBLX_BENCH_CHUNKS"])):
            c0, c1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            with torch.cuda.stream(stream):
                c0.record(stream)
                for _ in range(20):
                    step()
                c1.record(stream)
            torch.cuda.synchronize()
            cs.append(round(c0.elapsed_time(c1) / 20, 4))
        log(f"preload per-launch ms by 10s: {_PRELOAD_TRACE}")
        log(f"wall: preload end -> timed start {1e3 * (t0 - _T_PRE_END):.2f} ms")
        log(f"timed region {k_decode_ms:.4f} ms/launch; chunks of 20 after: {cs}")
    ms_per_step = elapsed * 1e3 / args.steps
    value = total_bytes / (elapsed / args.steps) / 2**30

    # roofline of the (only) decode kernel: algorithmic bytes per launch / its launch duration
    achieved = alg_bytes / (k_decode_ms * 1e-3) / 1e9
    mx = int(ln.max())
    kernel = ("k_decode_pipe<PipeSmall>" if mx <= PIPE_MAX_BLOCK else
              "k_decode_pipe<PipeLarge>" if mx <= PIPE_LARGE_MAX_BLOCK else "k_decode_tiles")
    traffic = None
    if os.path.exists(args.traffic_json):
        try:
            tj = json.load(open(args.traffic_json))
            if tj.get("kernel") == kernel and int(tj.get("blocks", -1)) == int(batch.nblk):
                traffic = tj.get("hbm_bytes_per_launch")
        except Exception:
            traffic = None

    if crc_info is not None:
        crc_info["fused_decode_verify"]["vs_decode_then_crc_GiB_per_s"] = \
            round(block_bytes / ((k_decode_ms + crc_info["ms"]) * 1e-3) / 2**30, 1)
    res = {
        "metric": "KV records/s + GiB/s of block bytes decoded, device-resident",
        "value": round(value, 3),
        "unit": "GiB/s",
        "records_per_s": round(total_recs / (elapsed / args.steps), 1),
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "preload": {"ms": args.preload_ms, "launches": n_pre,
                    "note": "untimed decode launches right before the W warmup steps (GPU clocks at their loaded state)"},
        "ms_per_step": round(ms_per_step, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u8",
        "data": "synthetic (seeded cfg2 generator, product Writer)",
        "config": {"workload": (f"cfg2: 4 KiB blocks" if args.block_size == 4096 else
                                f"cfg2 scheme with {args.block_size // 1024} KiB blocks (cfg4 leg)") +
                               ", 16 B keys / 64 B values, restart_interval=16, compression=none, device-resident decode",
                   "blocks_per_gpu": int(batch.nblk), "block_bytes_per_gpu": block_bytes,
                   "records_per_gpu": int(nrec), "key_bytes_per_gpu": int(kbytes), "value_bytes_per_gpu": int(vbytes),
                   "parallelism": f"block-sharded x{world}, no collective" + (
                       f" (rank-partitioned key space, synth.cfg2_shard; {total_bytes} block bytes over all ranks)"
                       if world > 1 else "") + (
                       f" -- DIAGNOSTIC: all {world} ranks on GPU 0, gloo collectives (rank path check, not scaling)"
                       if args.share_gpu else "")},
        "kernels_ms": {f"{kernel} (HIP events around the timed region / steps)": round(k_decode_ms, 4)},
        "host_enqueue_ms_per_step": round(t_enq * 1e3 / args.steps, 4),
        "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic,
                     "kernel": kernel, "alg_bytes_per_launch": int(alg_bytes),
                     "stream_copy_ceiling_GBs": round(ceiling, 1) if ceiling else None,
                     "stream_copy_kernel": f"mtblx_stream_copy variant {ceiling_variant}" if ceiling else None,
                     "frac_of_copy_ceiling": round(achieved / ceiling, 4) if ceiling else None},
    }
    if crc_info is not None:
        res["crc32c_verify"] = crc_info
    if not args.no_get and args.block_size == 4096 and not args.lib and not args.stamps:
        res["get_batch"] = get_leg(data, int(batch.nblk), rank)
    if not args.no_e2e and args.block_size == 4096 and not args.lib and not args.stamps:
        del out, ws
        torch.cuda.empty_cache()
        res["end_to_end"] = end_to_end(data, off, ln, int(nrec), int(kbytes), int(vbytes), args.e2e_passes, dist)
    if args.stamps:
        d = ws.buf[:128].cpu().numpy().view(np.uint64).astype(np.float64)
        names = ["copy:wait-ready", "w1:lookback+barrier", "w0:walk-loop", "w0:scan-publish",
                 "loader:dma-issue", "copy:barrier", "loader:dma-wait", "copy:copy", "w0:barrier",
                 "w0:trailers", "w0:interval-setup", "w1:barrier", "loader:barrier",
                 "copy:barrier-min-over-waves", "copy:prepare-max-over-waves"]
        ntl = max(d[15], 1)
        res["phase_cycles_per_tile"] = {n: round(d[k] / ntl, 1) for k, n in enumerate(names)}
        res["stamps_note"] = "diagnostic build (s_memtime, thread 0 of each workgroup), last step only; shares, not time"
        import ctypes as C
        from mtblx import _lib as mlib
        L = mlib.lib()
        if hasattr(L, "mtblx_dbg_timeline"):
            G = 1024
            tl = np.zeros((G, 16), np.uint64)
            if L.mtblx_dbg_timeline(tl.ctypes.data_as(C.POINTER(C.c_uint64)), G) == 0:
                tl_all = tl.copy()
                tl = tl[tl[:, 0] > 0].astype(np.int64)
                t0 = tl[:, 0].min()
                us = (tl[:, :6] - t0) / 100.0   # s_memrealtime ticks at 100 MHz
                res["timeline_us"] = {
                    n: {"min": round(float(us[:, k].min()), 2), "mean": round(float(us[:, k].mean()), 2),
                        "max": round(float(us[:, k].max()), 2)}
                    for k, n in enumerate(["entry", "preload", "first_walk", "iter0", "loop_end", "exit"])}
                res["timeline_us"]["tiles_per_wg"] = [int(tl[:, 6].min()), int(tl[:, 6].max())]
                le = us[:, 4]
                res["timeline_us"]["loop_end_pct"] = {q: round(float(np.percentile(le, q)), 2) for q in (10, 50, 90, 99)}
                res["timeline_us"]["loop_end_mean_by_tiles"] = {int(n): round(float(le[tl[:, 6] == n].mean()), 2)
                                                               for n in np.unique(tl[:, 6])}
                wg = np.nonzero(tl_all[:, 0] > 0)[0]
                res["timeline_us"]["loop_end_mean_by_xcd"] = [round(float(le[(wg % 8) == x].mean()), 2) for x in range(8)]
                res["timeline_us"]["latest_wgs"] = [int(x) for x in wg[np.argsort(-le)[:8]]]
                res["timeline_us"]["wgs"] = int(tl.shape[0])
                ux = (tl[:, 7:16] - t0) / 100.0     # penult, last look-back, copy0 done, copyN done, penult look-back, drains
                res["timeline_raw"] = [[round(float(x), 1) for x in us[i, [1, 3, 4, 5]]] + [int(tl[i, 6])] +
                                       [round(float(x), 1) for x in ux[i]]
                                       for i in range(us.shape[0])]

    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        res["cpu_baseline"] = cpu_baseline(data, off, ln, args.cpu_seconds)
    if rank == 0:
        print(json.dumps(res), flush=True)
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
