#!/usr/bin/env python3
"""profiles/r02/decode/: the decode kernel before (round-1 final) and after (current), from a
tools/rounds/gpu_profile_r02.sh run (gpurun_out/prof_r02).  Copies the kernel stats and PMC rows
of the decode kernel and writes summary.json / summary.md.  FETCH_SIZE is doubled (gfx950
reports half the bytes of wide streaming reads, MI355X_MICROARCH.md); both are KiB."""
import csv
import glob
import json
import os
import shutil

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "gpurun_out", "prof_r02")
DST = os.environ.get("PROF_DST") or os.path.join(ROOT, "profiles", "r02", "decode")
TRAFFIC = os.environ.get("PROF_TRAFFIC")   # write profiles/traffic.json (the bench's `traffic`) from cur_small


def rows(path):
    with open(path) as f:
        return list(csv.DictReader(f))


def bench_line(log):
    for l in open(log):
        if l.startswith("{"):
            return json.loads(l)
    return None


out = {}
os.makedirs(DST, exist_ok=True)
for tag in ("cur_small", "r01_small", "cur_large", "r01_large"):
    d = os.path.join(SRC, tag)
    if not os.path.isdir(d):
        continue
    st = [r for r in rows(os.path.join(d, "stats", "run_kernel_stats.csv")) if "k_decode_pipe" in r["Name"]]
    st.sort(key=lambda r: -float(r["TotalDurationNs"]))
    k = st[0]
    kname = k["Name"]
    shutil.copy(os.path.join(d, "stats", "run_kernel_stats.csv"), os.path.join(DST, f"{tag}_kernel_stats.csv"))
    rec = {"kernel": kname.split("(")[0], "calls": int(k["Calls"]), "avg_us": float(k["AverageNs"]) / 1e3}
    for p in ("fetch", "write", "sq1", "sq2"):
        rr = [r for r in rows(os.path.join(d, p, "run_counter_collection.csv")) if r["Kernel_Name"] == kname]
        with open(os.path.join(DST, f"{tag}_pmc_{p}.csv"), "w", newline="") as f:
            if rr:
                w = csv.DictWriter(f, fieldnames=list(rr[0].keys()))
                w.writeheader()
                w.writerows(rr)
        vals = {}
        for r in rr:   # the largest dispatch of each counter (full-batch launches)
            vals[r["Counter_Name"]] = max(vals.get(r["Counter_Name"], 0.0), float(r["Counter_Value"]))
        rec.update(vals)
    b = bench_line(os.path.join(SRC, f"{tag}_stats.log"))
    alg = b["roofline"]["alg_bytes_per_launch"] if b else None
    rec["alg_bytes"] = alg
    rec["bench_value_GiBs"] = b["value"] if b else None
    if "FETCH_SIZE" in rec and "WRITE_SIZE" in rec and alg:
        hbm = 2 * rec["FETCH_SIZE"] * 1024 + rec["WRITE_SIZE"] * 1024
        rec["hbm_bytes"] = hbm
        rec["traffic_ratio"] = hbm / alg
    rec["achieved_GBs"] = alg / (rec["avg_us"] * 1e-6) / 1e9 if alg else None
    rec["frac_of_8TBs"] = rec["achieved_GBs"] / 8000 if alg else None
    if "SQ_WAVE_CYCLES" in rec:
        wc = rec["SQ_WAVE_CYCLES"]
        rec["wait_any_frac"] = rec.get("SQ_WAIT_ANY", 0) / wc
        rec["wait_inst_any_frac"] = rec.get("SQ_WAIT_INST_ANY", 0) / wc
        rec["active_inst_any_frac"] = rec.get("SQ_ACTIVE_INST_ANY", 0) / wc
    out[tag] = rec
json.dump(out, open(os.path.join(DST, "summary.json"), "w"), indent=1)
if TRAFFIC and "cur_small" in out and out["cur_small"].get("hbm_bytes"):
    c = out["cur_small"]
    json.dump({"kernel": "k_decode_pipe<PipeSmall>", "blocks": 100000, "hbm_bytes_per_launch": c["hbm_bytes"],
               "alg_bytes_per_launch": c["alg_bytes"], "ratio": round(c["traffic_ratio"], 3),
               "source": os.path.relpath(DST, ROOT) + " (rocprofv3 --pmc FETCH_SIZE x2 + WRITE_SIZE, separate passes, "
                         "full-batch dispatches of the current kernel)"},
              open(os.path.join(ROOT, "profiles", "traffic.json"), "w"), indent=1)
keys = ["kernel", "avg_us", "achieved_GBs", "frac_of_8TBs", "traffic_ratio", "SQ_BUSY_CYCLES", "wait_any_frac",
        "wait_inst_any_frac", "active_inst_any_frac", "SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_LDS",
        "SQ_LDS_BANK_CONFLICT", "SQ_LDS_IDX_ACTIVE", "SQ_INSTS_VMEM_RD", "SQ_INSTS_VMEM_WR"]
with open(os.path.join(DST, "summary.md"), "w") as f:
    f.write("| | " + " | ".join(out) + " |\n|---|" + "---|" * len(out) + "\n")
    for k in keys:
        cells = []
        for t in out:
            v = out[t].get(k)
            cells.append(f"{v:.4g}" if isinstance(v, float) else str(v))
        f.write(f"| {k} | " + " | ".join(cells) + " |\n")
print(open(os.path.join(DST, "summary.md")).read())
