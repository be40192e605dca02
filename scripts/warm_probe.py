"""Diagnostic: why a 20-step bench reads below a 200-step one.  Times the cfg2 decode in
chunks of 20 launches (host sync between chunks), then 200 launches back to back, then
chunks again -- HIP events per chunk, in one process.
    python scripts/warm_probe.py"""
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "oxidized-mtbl_amd")]

from mtblx import codec, synth  # noqa: E402


def main():
    data, off, ln = synth.cfg2_file(100_000, block_size=4096, seed=synth.SEED_CFG2)
    batch = codec.DeviceBatch.from_host(data, off, ln)
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        ws = codec.Workspace(batch.nblk)
        probe = codec.DecodedBlocks(batch.nblk, 0, 0, 0)
        codec.count_blocks(batch, probe, ws, s)
    s.synchronize()
    nrec, kb, vb, _ = probe.totals_host()
    with torch.cuda.stream(s):
        out = codec.DecodedBlocks(batch.nblk, nrec, kb, vb)
    torch.cuda.synchronize()

    def chunk(k):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        with torch.cuda.stream(s):
            e0.record(s)
            for _ in range(k):
                codec.decode_into(batch, out, ws, s)
            e1.record(s)
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / k

    print("first 10 chunks of 20 (sync between):", [round(chunk(20), 4) for _ in range(10)], flush=True)
    print("200 back to back:", round(chunk(200), 4), flush=True)
    print("10 chunks of 20 after:", [round(chunk(20), 4) for _ in range(10)], flush=True)
    time.sleep(0.5)
    print("after 0.5 s idle, chunks of 20:", [round(chunk(20), 4) for _ in range(5)], flush=True)
    print("chunks of 5:", [round(chunk(5), 4) for _ in range(8)], flush=True)
    print("2000 back to back:", round(chunk(2000), 4), flush=True)


if __name__ == "__main__":
    main()
