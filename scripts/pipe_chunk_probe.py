"""End-to-end chunk-size sweep (diagnostic): the cfg2 file in pinned host memory, decoded by
mtblx_pipe_decode into host arrays with chunks of 8..128 MiB (bench.py's e2e leg uses 64 MiB),
5 passes per sample after a warm-up pass, two alternations; ms per pass and GiB/s."""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "oxidized-mtbl_amd"))
import torch  # noqa: E402
from mtblx import codec, pipe, synth  # noqa: E402

data, off, ln = synth.cfg2_file(100_000)
nr, kb, vb, _ = codec.decode_blocks(codec.DeviceBatch.from_host(data, off, ln)).totals_host()
torch.cuda.synchronize()
block_bytes = int(ln.sum(dtype=np.uint64))
out = pipe.HostOutputs(off.size, nr, kb, vb)
pipe.register(data)
sizes = [int(x) for x in (sys.argv[1:] or ["8", "16", "32", "64", "128"])]
pipes = {m: pipe.HostPipe(chunk_bytes=m << 20, max_blocks=1 << 16, threads=16, device_snappy=False) for m in sizes}
res = {m: [] for m in sizes}
try:
    for rnd in range(2):
        for m in (sizes if rnd == 0 else sizes[::-1]):
            p = pipes[m]
            p.decode(data, off, ln, out, compression=0)
            t0 = time.perf_counter()
            for _ in range(5):
                st = p.decode(data, off, ln, out, compression=0)
            el = (time.perf_counter() - t0) / 5
            tot = out.totals
            assert int(tot[0]) == nr and int(tot[1]) == kb and int(tot[2]) == vb and int(tot[3]) == 0
            res[m].append(el)
            print(f"chunk {m:4d} MiB: {el * 1e3:7.3f} ms/pass = {block_bytes / el / 2**30:6.2f} GiB/s ({int(st.chunks)} chunks)", flush=True)
finally:
    pipe.unregister(data)
for m in sizes:
    b = min(res[m])
    print(f"best chunk {m:4d} MiB: {b * 1e3:7.3f} ms/pass = {block_bytes / b / 2**30:6.2f} GiB/s")
