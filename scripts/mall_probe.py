"""Decode + verify in chunks (diagnostic): does the second pass over a chunk's block bytes come
from the Infinity Cache (MALL, 256 MB) when the two passes run chunk by chunk?  cfg2 batch
(100 000 x 4 KiB = 402 MB).  For each library (argv; "prod" = the product libmtblx.so, else
build/libmtblx_<name>.so) in its own child process, HIP events around 30 repetitions of:
  decode, crc            the whole batch, one pass each (the product's two-launch verify)
  dc<K>, cd<K>           K chunks, decode then crc / crc then decode, chunk by chunk
  d<K>, c<K>             K chunks of one pass alone
Outputs go to per-chunk buffers (timing only; no bases carried across chunks)."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r'''
import os, sys, json, time, ctypes as C
sys.path.insert(0, os.path.join(%r, "oxidized-mtbl_amd"))
import torch
from mtblx import codec, synth, _lib
L = _lib.lib()
data, off, ln = synth.cfg2_file(int(os.environ.get("AB_BLOCKS", "100000")))
full = codec.DeviceBatch.from_host(data, off, ln)
s = torch.cuda.Stream()
def sub(lo, hi):
    return codec.DeviceBatch(full.data, full.blk_off[lo:hi], full.blk_len[lo:hi], full.max_blk_len)
def make(b):
    ws = codec.Workspace(b.nblk)
    with torch.cuda.stream(s):
        out = codec.decode_blocks(b, stream=s)
    crc = torch.zeros(b.nblk, dtype=torch.int32, device="cuda")
    bad = torch.zeros(b.nblk, dtype=torch.uint8, device="cuda")
    return [b, out, ws, crc, bad]
def dec(u):
    codec.decode_into(u[0], u[1], u[2], s)
def crc(u):
    rc = L.mtblx_crc32c_blocks(C.byref(u[0].cstruct()), C.c_void_p(u[3].data_ptr()), C.c_void_p(u[4].data_ptr()), 1,
                               C.c_void_p(s.cuda_stream))
    assert rc == 0
def timed(fn, reps):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    with torch.cuda.stream(s):
        e0.record(s)
        for _ in range(reps):
            fn()
        e1.record(s)
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps
n = full.nblk
units = {1: [make(full)]}
for K in (2, 3, 4, 6, 8):
    cut = [n * i // K for i in range(K + 1)]
    units[K] = [make(sub(cut[i], cut[i + 1])) for i in range(K)]
torch.cuda.synchronize()
u1 = units[1][0]
t0 = time.perf_counter()
while time.perf_counter() - t0 < 0.3:
    timed(lambda: dec(u1), 10)
res = {}
res["decode"] = timed(lambda: dec(u1), 30)
res["crc"] = timed(lambda: crc(u1), 30)
res["dc1"] = timed(lambda: (dec(u1), crc(u1)), 30)
for K in (2, 3, 4, 6, 8):
    us = units[K]
    res["d%%d" %% K] = timed(lambda: [dec(u) for u in us], 30)
    res["c%%d" %% K] = timed(lambda: [crc(u) for u in us], 30)
    res["dc%%d" %% K] = timed(lambda: [(dec(u), crc(u)) for u in us], 30)
    res["cd%%d" %% K] = timed(lambda: [(crc(u), dec(u)) for u in us], 30)
bytes_ = int(ln.astype("int64").sum())
res = {k: round(v, 4) for k, v in res.items()}
res["GiBps_best"] = round(bytes_ / (min(v for k, v in res.items() if k.startswith(("dc", "cd"))) * 1e-3) / 2**30, 1)
print(json.dumps(res))
''' % ROOT

libs = sys.argv[1:] or ["prod"]
for rnd in range(2):
    for lib in libs:
        env = dict(os.environ)
        if lib != "prod":
            env["MTBLX_LIB"] = os.path.join(ROOT, "oxidized-mtbl_amd", "build", f"libmtblx_{lib}.so")
        r = subprocess.run([sys.executable, "-c", CHILD], env=env, capture_output=True, text=True, timeout=300)
        if r.returncode != 0:
            print(lib, r.stderr[-2000:])
            sys.exit(1)
        print(lib, r.stdout.strip().splitlines()[-1], flush=True)
