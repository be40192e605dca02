#!/usr/bin/env python3
"""profiles/r02/cfg3/: k_decode_pipe<PipeLarge> and k_encode on one cfg3 chunk, from a
tools/rounds/gpu_profile_cfg3.sh run (gpurun_out/prof_cfg3).  Per kernel: average duration, PMC bytes
per launch (FETCH_SIZE x 2, the gfx950 correction of MI355X_MICROARCH.md, + WRITE_SIZE; both KiB)
against the bench's algorithmic bytes per launch, and SQ wait / active fractions."""
import csv
import glob
import json
import os
import shutil

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "gpurun_out", "prof_cfg3")
DST = os.environ.get("CFG3_DST") or os.path.join(ROOT, "profiles", "r02", "cfg3")


def rows(pattern):
    out = []
    for f in glob.glob(os.path.join(SRC, pattern), recursive=True):
        with open(f) as fh:
            out += list(csv.DictReader(fh))
    return out


def bench_line(log):
    for l in open(log):
        if l.startswith("{"):
            return json.loads(l)
    return None


os.makedirs(DST, exist_ok=True)
line = bench_line(os.path.join(SRC, "stats.log"))
alg = {"decode": line["roofline"]["decode"]["alg_bytes"], "encode": line["roofline"]["encode"]["alg_bytes"]}
stats = rows("stats/**/*kernel_stats.csv")
shutil.copy(glob.glob(os.path.join(SRC, "stats", "**", "*kernel_stats.csv"), recursive=True)[0],
            os.path.join(DST, "kernel_stats.csv"))
summary = {"bench_line": {k: line.get(k) for k in ("metric", "value", "unit", "encode_GiB_per_s", "config", "roofline")}}
for role, key in (("decode", "k_decode_pipe"), ("encode", "k_encode")):
    st = [r for r in stats if key in r["Name"]]
    st.sort(key=lambda r: -float(r["TotalDurationNs"]))
    k = st[0]
    name = k["Name"]
    rec = {"kernel": name.split("(")[0], "calls": int(k["Calls"]), "avg_us": float(k["AverageNs"]) / 1e3}
    rec["alg_bytes_per_launch"] = alg[role]
    rec["achieved_GBs"] = alg[role] / (rec["avg_us"] * 1e-6) / 1e9
    rec["frac_of_8TBs"] = rec["achieved_GBs"] / 8000.0
    pm = {}
    for p in ("fetch", "write", "sq"):
        rr = [r for r in rows(f"{p}/**/*counter_collection.csv") if r["Kernel_Name"] == name]
        per = {}
        for r in rr:
            per.setdefault((r["Dispatch_Id"], r["Counter_Name"]), 0.0)
            per[(r["Dispatch_Id"], r["Counter_Name"])] += float(r["Counter_Value"])
        byc = {}
        for (d, c), v in per.items():
            byc.setdefault(c, []).append(v)
        for c, v in byc.items():
            pm[c] = sum(v) / len(v)
        if rr:
            shutil.copy(glob.glob(os.path.join(SRC, p, "**", "*counter_collection.csv"), recursive=True)[0],
                        os.path.join(DST, f"pmc_{p}.csv"))
    rec["pmc"] = pm
    if "FETCH_SIZE" in pm and "WRITE_SIZE" in pm:
        hbm = (2 * pm["FETCH_SIZE"] + pm["WRITE_SIZE"]) * 1024
        rec["hbm_bytes_per_launch"] = hbm
        rec["traffic_ratio"] = hbm / alg[role]
    if "SQ_WAVE_CYCLES" in pm:
        for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY"):
            if c in pm:
                rec[c.lower() + "_frac"] = pm[c] / pm["SQ_WAVE_CYCLES"]
    summary[role] = rec
json.dump(summary, open(os.path.join(DST, "summary.json"), "w"), indent=1)
for role in ("decode", "encode"):
    r = summary[role]
    print(role, r["kernel"], f"{r['avg_us']:.1f} us", f"{r['achieved_GBs']:.0f} GB/s", f"frac {r['frac_of_8TBs']:.3f}",
          f"traffic {r.get('traffic_ratio', float('nan')):.3f}", f"wait {r.get('sq_wait_any_frac', float('nan')):.2f}")
