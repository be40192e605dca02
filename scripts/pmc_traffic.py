#!/usr/bin/env python3
"""Turn a gpu_profile.sh run (gpurun_out/prof_<tag>/) into the committed profile evidence:

profiles/<tag>/kernel_stats.csv     rocprofv3 --kernel-trace --stats summary
profiles/<tag>/bench.json           the bench line of that session
profiles/<tag>/pmc_*.csv            per-dispatch FETCH_SIZE / WRITE_SIZE rows of the decode kernel
profiles/traffic.json               HBM bytes per decode launch, read by bench.py as roofline.traffic

FETCH_SIZE is doubled: on gfx950 it reports exactly half the bytes of wide (16 B/lane) streaming
reads (/opt/skills/guides/MI355X_MICROARCH.md, HBM section); WRITE_SIZE is exact for 16 B/lane stores.
Both are in KiB (rocprofv3 derived counters) -> x1024.
"""
import csv
import glob
import json
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def rows(pattern):
    out = []
    for f in glob.glob(pattern, recursive=True):
        with open(f) as fh:
            out += list(csv.DictReader(fh))
    return out


# the product decode of the cfg2 batch: k_decode_pipe<PipeSmall> (not the fused-verify variant)
KERNEL_MATCH = "PipeCfg<49152, 3, 16, 56, false"


def counter(d, name, kernel):
    vals = [float(r["Counter_Value"]) for r in rows(os.path.join(d, "**", "*counter_collection.csv"))
            if r.get("Counter_Name") == name and KERNEL_MATCH in r.get("Kernel_Name", "")]
    # the full-batch launches (the bench's end-to-end section decodes smaller chunks)
    top = max(vals) if vals else 0.0
    return [v for v in vals if v >= 0.9 * top]


def main():
    tag = sys.argv[1] if len(sys.argv) > 1 else "r01"
    src = os.path.join(ROOT, "gpurun_out", f"prof_{tag}")
    dst = os.path.join(ROOT, "profiles", tag)
    os.makedirs(dst, exist_ok=True)
    stats = glob.glob(os.path.join(src, "stats", "**", "*kernel_stats.csv"), recursive=True)
    if stats:
        shutil.copy(stats[0], os.path.join(dst, "kernel_stats.csv"))
    bench_log = os.path.join(ROOT, "gpurun_out", "bench.log")
    if os.path.exists(bench_log):
        lines = [ln for ln in open(bench_log) if ln.startswith("{")]
        if lines:
            open(os.path.join(dst, "bench.json"), "w").write(lines[-1])
    bench = json.loads(open(os.path.join(dst, "bench.json")).read()) if os.path.exists(
        os.path.join(dst, "bench.json")) else {}
    kernel = bench.get("roofline", {}).get("kernel", "k_decode_pipe")
    fetch = counter(os.path.join(src, "fetch"), "FETCH_SIZE", kernel)
    write = counter(os.path.join(src, "write"), "WRITE_SIZE", kernel)
    for name, d in (("fetch", "FETCH_SIZE"), ("write", "WRITE_SIZE")):
        sel = [r for r in rows(os.path.join(src, name, "**", "*counter_collection.csv"))
               if r.get("Counter_Name") == d and KERNEL_MATCH in r.get("Kernel_Name", "")]
        if sel:
            with open(os.path.join(dst, f"pmc_{name}.csv"), "w", newline="") as fh:
                w = csv.DictWriter(fh, fieldnames=list(sel[0].keys()))
                w.writeheader()
                w.writerows(sel)
    if not fetch or not write:
        print("no PMC rows for", kernel)
        return
    # full-batch launches only (see counter); the count probe moves no key/value bytes
    f = sum(fetch[-5:]) / len(fetch[-5:]) * 1024.0
    w = sum(write[-5:]) / len(write[-5:]) * 1024.0
    alg = bench.get("roofline", {}).get("alg_bytes_per_launch")
    res = {
        "kernel": kernel,
        "blocks": bench.get("config", {}).get("blocks_per_gpu"),
        "fetch_size_raw_bytes": f,
        "fetch_bytes_corrected": 2.0 * f,
        "write_bytes": w,
        "hbm_bytes_per_launch": 2.0 * f + w,
        "alg_bytes_per_launch": alg,
        "traffic_over_alg": (2.0 * f + w) / alg if alg else None,
        "source": f"profiles/{tag}/pmc_fetch.csv, pmc_write.csv (rocprofv3 --pmc, separate passes)",
        "note": "FETCH_SIZE x2 (gfx950 wide-read correction), KiB -> bytes; mean of the last 5 full-batch dispatches",
    }
    json.dump(res, open(os.path.join(ROOT, "profiles", "traffic.json"), "w"), indent=1)
    json.dump(res, open(os.path.join(dst, "traffic.json"), "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
