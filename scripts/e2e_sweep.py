"""Diagnostic: end-to-end pipe rate vs chunk size, beside the raw pinned PCIe copy rates."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "oxidized-mtbl_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402


def pcie():
    n = 400 << 20
    h = torch.empty(n, dtype=torch.uint8).pin_memory()
    h2 = torch.empty(n, dtype=torch.uint8).pin_memory()
    d = torch.empty(n, dtype=torch.uint8, device="cuda")
    d2 = torch.empty(n, dtype=torch.uint8, device="cuda")
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    for _ in range(2):
        d.copy_(h, non_blocking=True)
        h2.copy_(d2, non_blocking=True)
    torch.cuda.synchronize()
    r = {}
    t = time.perf_counter()
    for _ in range(5):
        d.copy_(h, non_blocking=True)
    torch.cuda.synchronize()
    r["h2d_GBs"] = 5 * n / (time.perf_counter() - t) / 1e9
    t = time.perf_counter()
    for _ in range(5):
        h2.copy_(d2, non_blocking=True)
    torch.cuda.synchronize()
    r["d2h_GBs"] = 5 * n / (time.perf_counter() - t) / 1e9
    t = time.perf_counter()
    for _ in range(5):
        with torch.cuda.stream(s1):
            d.copy_(h, non_blocking=True)
        with torch.cuda.stream(s2):
            h2.copy_(d2, non_blocking=True)
    torch.cuda.synchronize()
    r["bidir_GBs_each"] = 5 * n / (time.perf_counter() - t) / 1e9
    return r


def main():
    from mtblx import pipe, synth
    data, off, ln = synth.cfg2_file(100_000)
    nrec = int(synth.cfg2_file.last_block_nrec.sum())
    out = pipe.HostOutputs(off.size, nrec, 16 * nrec, 64 * nrec)
    pipe.register(data)
    res = {"pcie": pcie(), "sweep": []}
    bb = int(ln.sum())
    for chunk in (4 << 20, 8 << 20, 16 << 20, 32 << 20, 64 << 20):
        for thr in (4, 16):
            p = pipe.HostPipe(chunk_bytes=chunk, threads=thr)
            p.decode(data, off, ln, out)
            t = time.perf_counter()
            for _ in range(5):
                st = p.decode(data, off, ln, out)
            el = (time.perf_counter() - t) / 5
            res["sweep"].append({"chunk_MiB": chunk >> 20, "threads": thr, "GiB_per_s": round(bb / el / 2**30, 2),
                                 "ms": round(el * 1e3, 3), "chunks": st.chunks})
            del p
    pipe.unregister(data)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
