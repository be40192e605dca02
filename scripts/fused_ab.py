"""A/B of decode builds on the cfg2 bench batch (diagnostic): for each library (argv; "prod" =
the product libmtblx.so) in its own child process, HIP events around 50 launches after a warm
loop: the plain decode, the fused decode + verify (k_decode_pipe<PipeSmallV>) and decode then
k_crc32c_blocks; bad = blocks the verify flagged (ablation builds flag blocks by construction)."""
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
data, off, ln = synth.cfg2_file(int(os.environ.get("AB_BLOCKS", "100000")))
batch = codec.DeviceBatch.from_host(data, off, ln)
s = torch.cuda.Stream()
def timed(fn, reps):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    with torch.cuda.stream(s):
        e0.record(s)
        for _ in range(reps):
            fn()
        e1.record(s)
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps
ws = codec.Workspace(batch.nblk)
with torch.cuda.stream(s):
    out = codec.decode_blocks(batch, stream=s)
torch.cuda.synchronize()
dec = lambda: codec.decode_into(batch, out, ws, s)
t0 = time.perf_counter()
while time.perf_counter() - t0 < 0.2:
    timed(dec, 10)
res = {}
res["decode_ms"] = timed(dec, 50)
vbad = torch.zeros(batch.nblk, dtype=torch.uint8, device="cuda")
for name, fused in (("fused_ms", True), ("decode_then_crc_ms", False)):
    g = lambda: codec.decode_verify_into(batch, out, ws, None, vbad, True, s, fused=fused)
    for _ in range(20):
        g()
    vbad.zero_()
    res[name] = timed(g, 50)
    res[name.replace("_ms", "_bad")] = int((vbad != 0).sum().item())
res = {k: (round(v, 4) if isinstance(v, float) else v) for k, v in res.items()}
print(json.dumps(res))
''' % ROOT

res = {}
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
        d = json.loads(r.stdout.strip().splitlines()[-1])
        res.setdefault(lib, []).append(d)
        print(lib, d, flush=True)
print(json.dumps(res))
