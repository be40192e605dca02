"""Timing of the CRC-32C kernel over the cfg2 bench batch: each run in its own child process
(argv names runs: "kernel" sets MTBLX_CRC_KERNEL, "kernel@lib" also MTBLX_LIB = that library,
e.g. a diagnostic variant; "!" at the end: an ablation whose checksums are wrong by design),
HIP events around 50 launches after a 200 ms preload, two alternations; also decode + verify.
Round 3 measured kernels 0-7 with it (profiles/r03/crc_ab.txt); only kernel 0 remains."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r'''
import os, sys, json, time
sys.path.insert(0, os.path.join(%r, "oxidized-mtbl_amd"))
import torch
from mtblx import codec, synth
data, off, ln = synth.cfg2_file(100_000)
batch = codec.DeviceBatch.from_host(data, off, ln)
s = torch.cuda.Stream()
crc, bad = codec.crc32c_blocks(batch, framed=True, stream=s)
torch.cuda.synchronize()
ABL = os.environ.get("CRC_AB_ABLATION") == "1"
assert ABL or int(bad.sum().item()) == 0
def timed(fn, reps):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    with torch.cuda.stream(s):
        e0.record(s)
        for _ in range(reps):
            fn()
        e1.record(s)
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps
f = lambda: codec.crc32c_blocks(batch, framed=True, stream=s)
t0 = time.perf_counter()
while time.perf_counter() - t0 < 0.2:
    timed(f, 10)
crc_ms = timed(f, 50)
ws = codec.Workspace(batch.nblk)
with torch.cuda.stream(s):
    out = codec.decode_blocks(batch, stream=s)
torch.cuda.synchronize()
vbad = torch.zeros(batch.nblk, dtype=torch.uint8, device="cuda")
g = lambda: codec.decode_verify_into(batch, out, ws, None, vbad, True, s, fused=False)
for _ in range(20):
    g()
dv_ms = timed(g, 50)
assert ABL or int(vbad.sum().item()) == 0
print(json.dumps({"crc_ms": round(crc_ms, 4), "decode_verify_ms": round(dv_ms, 4),
                  "crc_GiBs": round(float(ln.sum()) / crc_ms / 1e-3 / 2**30, 1),
                  "decode_verify_GiBs": round(float(ln.sum()) / dv_ms / 1e-3 / 2**30, 1)}))
''' % ROOT

res = {}
for rnd in range(2):
    for k in sys.argv[1:] or ["0", "1", "2"]:
        name, _, lib = k.rstrip("!").partition("@")
        env = dict(os.environ, MTBLX_CRC_KERNEL=name, CRC_AB_ABLATION="1" if k.endswith("!") else "0")
        if lib:
            env["MTBLX_LIB"] = os.path.abspath(lib)
        r = subprocess.run([sys.executable, "-c", CHILD], env=env, capture_output=True, text=True, timeout=300)
        if r.returncode != 0:
            print(r.stderr[-2000:])
            sys.exit(1)
        d = json.loads(r.stdout.strip().splitlines()[-1])
        res.setdefault(k, []).append(d)
        print(k, d, flush=True)
print(json.dumps(res))
