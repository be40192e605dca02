# diagnostic: device vs oracle per-block counts on a small cfg2 batch
import sys, os
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "oxidized-mtbl_amd"), os.path.join(ROOT, "oracle")]
import numpy as np, torch, pyoracle
from mtblx import codec, synth
nb = int(sys.argv[1]) if len(sys.argv) > 1 else 3000
data, off, ln = synth.cfg2_file(nb)
orc = pyoracle.decode_blocks(data, off, ln)
batch = codec.DeviceBatch.from_host(data, off, ln)
out = codec.decode_blocks(batch)
torch.cuda.synchronize()
h = out.to_host()
print("totals dev", h.totals, "orc", int(orc.nrec.sum()), orc.keys.size, orc.vals.size)
bad = np.nonzero(h.nrec != orc.nrec)[0]
print("nrec mismatches", bad.size, bad[:20], h.nrec[bad[:20]], orc.nrec[bad[:20]])
badb = np.nonzero(h.rec_base != orc.rec_base)[0]
print("rec_base mismatches", badb.size, badb[:10], h.rec_base[badb[:10]], orc.rec_base[badb[:10]])
print("status", np.unique(h.status, return_counts=True))
