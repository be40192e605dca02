"""Writer block cut (mtblx_encode_plan) on one cfg3 chunk: wall ms per call after a warm-up
call, for the parallel planner (default) and the serial walk (MTBLX_PLAN=serial, read at the
library's first call).  Prints one JSON line."""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "oxidized-mtbl_amd"))
from mtblx import encode, synth  # noqa: E402


def main():
    nrec = int(sys.argv[1]) if len(sys.argv) > 1 else 6_593_024
    nsh = int(sys.argv[2]) if len(sys.argv) > 2 else 64
    reps = 5
    recs, _ = synth.cfg3_records_device(nrec, seed=synth.SEED_CFG3)
    cuts = torch.linspace(0, nrec, nsh + 1, device="cuda").to(torch.int64)
    blk = encode.plan(recs, 65536, 16, shard_rec=cuts)
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        b2 = encode.plan(recs, 65536, 16, shard_rec=cuts)
        torch.cuda.synchronize()
        ts.append((time.perf_counter() - t0) * 1e3)
    assert torch.equal(blk, b2)
    print(json.dumps({"probe": "mtblx_encode_plan", "mode": os.environ.get("MTBLX_PLAN", "parallel"), "records": nrec,
                      "shards": nsh, "blocks": int(blk.numel()) - 1, "ms": [round(t, 2) for t in ts],
                      "ms_min": round(min(ts), 2)}))


if __name__ == "__main__":
    main()
