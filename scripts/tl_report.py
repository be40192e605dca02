"""Summarise the per-workgroup timeline a `bench.py --stamps` run printed (diagnostic)."""
import json
import sys

import numpy as np

for l in open(sys.argv[1]):
    if l.startswith('{'):
        d = json.loads(l)
print("ms_per_step", d["ms_per_step"], json.dumps({k: v for k, v in d["timeline_us"].items()}))
r = np.array(d["timeline_raw"])
g = np.arange(len(r))
le, ex, n = r[:, 2], r[:, 3], r[:, 4]
print("drain exit-loop_end: mean %.1f max %.1f" % ((ex - le).mean(), (ex - le).max()))
for t in sorted(set(n.astype(int))):
    m = n == t
    print(t, m.sum(), "loop_end mean %.1f min %.1f max %.1f" % (le[m].mean(), le[m].min(), le[m].max()))
for x in range(8):
    m = g % 8 == x
    print("xcd", x, "loop_end/tiles mean %.2f" % (le[m] / n[m]).mean(), "max %.1f" % le[m].max())
