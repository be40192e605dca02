"""Diagnostic: decode totals across repeated calls (run under rocprofv3 --pmc and without)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "oxidized-mtbl_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from mtblx import codec, synth  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 2000
data, off, ln = synth.cfg2_file(n)
exp = int(synth.cfg2_file.last_block_nrec.sum())
batch = codec.DeviceBatch.from_host(data, off, ln)
ws = codec.Workspace(batch.nblk)
probe = codec.DecodedBlocks(batch.nblk, 0, 0, 0)
codec.count_blocks(batch, probe, ws)
torch.cuda.synchronize()
print("probe", probe.totals_host(), "expected nrec", exp, "ws hdr", ws.buf[128:144].cpu().numpy().view(np.uint32))
nr, kb, vb, _ = probe.totals_host()
out = codec.DecodedBlocks(batch.nblk, max(nr, exp), max(kb, 16 * exp), max(vb, 64 * exp))
for i in range(4):
    out.totals.zero_()
    codec.decode_into(batch, out, ws)
    torch.cuda.synchronize()
    st = out.status[: batch.nblk].cpu().numpy()
    print("decode", i, out.totals_host(), "status!=0:", int((st != 0).sum()), "nrec sum",
          int(out.nrec[: batch.nblk].cpu().numpy().view(np.uint32).sum()),
          "ws hdr", ws.buf[128:144].cpu().numpy().view(np.uint32))
