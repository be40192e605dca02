"""Diagnostic: k_crc32c_blocks over the cfg2 bench batch, N launches (for rocprofv3 runs)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "oxidized-mtbl_amd"))
import torch  # noqa: E402

from mtblx import codec, synth  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 100_000
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 20
data, off, ln = synth.cfg2_file(n)
batch = codec.DeviceBatch.from_host(data, off, ln)
for _ in range(reps):
    crc, bad = codec.crc32c_blocks(batch, framed=True)
torch.cuda.synchronize()
print("bad", int(bad.sum().item()))
