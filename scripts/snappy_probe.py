"""Diagnostic: device snappy decompression of the cfg5 stored blocks (cfg2 records written with
CompressionType::Snappy), timed with HIP events; run under rocprofv3 for kernel stats / PMC.
    python scripts/snappy_probe.py [--blocks N] [--reps R]"""
import argparse
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "oxidized-mtbl_amd")]

from mtblx import _lib, codec, synth  # noqa: E402
from mtblx.writer import Writer  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--blocks", type=int, default=100_000)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--compressible", action="store_true", help="cfg1-style repeated values instead")
    ap.add_argument("--tile", type=int, default=1, help="the generated file's blocks this many times over")
    a = ap.parse_args()
    t0 = time.time()
    w = Writer(4096, 16, 1)
    if a.compressible:
        for k, v in synth.cfg1_records(a.blocks * 20):
            w.insert(k, v)
        z = np.frombuffer(w.into_inner(), np.uint8).copy()
    else:
        per = (4096 - 64) // 79
        n = a.blocks * per
        keys, vals, kl, vl = synth.cfg2_arrays(n)
        w.insert_batch(keys, np.arange(1, n + 1, dtype=np.uint64) * np.uint64(kl), vals,
                       np.arange(1, n + 1, dtype=np.uint64) * np.uint64(vl))
        z = w.into_inner_np()
    zoff, zln = w.block_dir
    if a.tile > 1:   # bench.py compressible_snappy's 100 000-block batch: the file tiled
        zoff = np.concatenate([zoff.astype(np.uint64) + np.uint64(i * z.size) for i in range(a.tile)])
        zln = np.tile(zln, a.tile)
        z = np.tile(z, a.tile)
    print(f"generated {zoff.size} blocks, {int(zln.sum()) / 2**20:.1f} MiB stored in {time.time() - t0:.1f}s",
          flush=True)
    zb = codec.SnappyBatch.from_host(z, zoff, zln)
    lay = codec.SnappyLayout(zb.nblk)
    codec.snappy_dir(zb, lay)
    torch.cuda.synchronize()
    tot = lay.totals.cpu().numpy().view(np.uint64)
    dst = torch.zeros(int(tot[0]) + 16, dtype=torch.uint8, device="cuda")
    st = torch.zeros(zb.nblk, dtype=torch.int32, device="cuda")
    dl = torch.zeros(zb.nblk, dtype=torch.int32, device="cuda")
    s = torch.cuda.current_stream()
    # ~40 ms of untimed launches first: the GPU drops its clocks when idle (bench.py _preload)
    t_pre = time.perf_counter()
    while time.perf_counter() - t_pre < 0.04:
        for _ in range(5):
            codec.snappy_decompress_into(zb, lay, dst, st, dl, int(tot[1]), s)
        torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(s)
    for _ in range(a.reps):
        codec.snappy_decompress_into(zb, lay, dst, st, dl, int(tot[1]), s)
    e1.record(s)
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / a.reps
    out_bytes = int(dl.sum().item())
    print(f"decompress {ms:.4f} ms  {out_bytes / ms / 1e6:.1f} GB/s out  stored {int(zln.sum()) / ms / 1e6:.1f} GB/s in"
          f"  bad={int((st != 0).sum().item())}", flush=True)
    L = _lib.lib()
    if hasattr(L, "mtblx_snap_debug"):   # the snapstamps diagnostic build
        import ctypes as C
        dbg = (C.c_uint64 * 8)()
        L.mtblx_snap_debug(dbg, 1)
        codec.snappy_decompress_into(zb, lay, dst, st, dl, int(tot[1]), s)
        torch.cuda.synchronize()
        L.mtblx_snap_debug(dbg, 0)
        if os.environ.get("MTBLX_SNAPPY_KERNEL") == "lanes":   # k_snappy_lanes' per-path counters
            it = max(int(dbg[0]), 1)
            names = ["iterations", "decode", "literal(window)", "literal(HBM)", "ring copy", "far copy",
                     "overlapping copy", "window reload"]
            print("lanes: wave iterations %d; share of iterations where any lane took: %s" % (
                it, ", ".join("%s %.3f" % (names[k], dbg[k] / it) for k in range(1, 8))), flush=True)
            return
        if os.environ.get("MTBLX_SNAPPY_KERNEL") == "waves":   # k_snappy_waves' per-phase stamps
            nb = max(int(dbg[5]), 1)
            print("waves per block: stage %.0f  chain %.0f  records %.0f  literals %.0f  copy rounds %.0f (%.1f rounds)"
                  "  output %.0f cycles" % (dbg[0] / nb, dbg[1] / nb, dbg[2] / nb, dbg[3] / nb, dbg[4] / nb,
                                            dbg[6] / nb, dbg[7] / nb), flush=True)
            return
        nb = max(int(dbg[5]), 1)
        print("per block: cycles %.0f  in flush %.0f  store %.0f  elements %.1f  flushes %.1f  restages %.2f  steps %.1f"
              % (dbg[0] / nb, dbg[1] / nb, dbg[2] / nb, dbg[3] / nb, dbg[4] / nb, dbg[6] / nb, dbg[7] / nb), flush=True)


if __name__ == "__main__":
    main()
