#!/usr/bin/env python3
"""profiles/<round>/<tag>/ from a scripts/gpu_evidence.sh run (gpurun_out/<round>/ev_<tag>/; ROUND, default r04).

driver/: the driver's command (`bench.py --gpus 1 --steps 20 --warmup 5`) under
  rocprofv3 --kernel-trace --stats.  The timed steps are the LAST K launches of the bench's
  decode kernel on the decode stream (the bench's end-to-end legs run on the pipe's own
  streams; everything else on the decode stream precedes the preload / warmup / timed steps).
  Writes timed_launches.csv (per launch: duration, achieved GB/s, frac of 8 TB/s) and
  summary.json (their mean against the bench line's HIP-event figure).
fetch/, write/: FETCH_SIZE (x2, gfx950 wide-read correction) and WRITE_SIZE per full-batch
  dispatch of the decode kernel -> summary.json `traffic`, and profiles/traffic.json (what
  bench.py reports as roofline.traffic).
cfg2_845k/, cfg4/: per-launch durations of the cfg2 batch at the cfg4 4 KiB leg's size and of
  the cfg4 legs (the cfg4 4 KiB-leg gap)."""
import csv
import glob
import json
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PEAK = 8000.0
RND = os.environ.get("ROUND", "r04")
SMALL = ", 3, 16, 56, false"   # PipeSmall (any staging size: 49 152 before round 6, 49 664 since)
LARGE = "PipeCfg<65664, 2, 2, 64, false"


def rows(pattern):
    out = []
    for f in sorted(glob.glob(pattern, recursive=True)):
        with open(f) as fh:
            out += list(csv.DictReader(fh))
    return out


def bench_line(log):
    if not os.path.exists(log):
        return None
    for ln in open(log):
        if ln.startswith("{"):
            return json.loads(ln)
    return None


def launches(d, match):
    """decode launches of kernel `match` in dispatch order -> {stream: [(dispatch, ns)]}"""
    by = {}
    for r in rows(os.path.join(d, "**", "*kernel_trace.csv")):
        if "k_decode_pipe" in r["Kernel_Name"] and match in r["Kernel_Name"]:
            ns = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
            by.setdefault(r["Stream_Id"], []).append((int(r["Dispatch_Id"]), ns, int(r["Start_Timestamp"])))
    for v in by.values():
        v.sort()
    return by


def main():
    tag = sys.argv[1] if len(sys.argv) > 1 else "run"
    src = os.path.join(ROOT, "gpurun_out", RND, f"ev_{tag}")
    dst = os.path.join(ROOT, "profiles", RND, os.environ.get("PROF_NAME", tag))
    os.makedirs(dst, exist_ok=True)
    summ = {}
    # ---- the driver command
    b = bench_line(os.path.join(src, "driver_trace.log"))
    if b:
        json.dump(b, open(os.path.join(dst, "bench_line.json"), "w"), indent=1)
        K = int(b["steps"])
        alg = int(b["roofline"]["alg_bytes_per_launch"])
        by = launches(os.path.join(src, "driver"), SMALL)
        stream = max(by, key=lambda s: len(by[s]))
        timed = by[stream][-K:]
        with open(os.path.join(dst, "timed_launches.csv"), "w", newline="") as fh:
            w = csv.writer(fh)
            w.writerow(["dispatch_id", "duration_us", "achieved_GBs", "frac_of_8TBs"])
            for did, ns, _ in timed:
                w.writerow([did, round(ns / 1e3, 2), round(alg / ns, 1), round(alg / ns / PEAK, 4)])
        avg_ns = sum(ns for _, ns, _ in timed) / len(timed)
        span_ns = timed[-1][2] + timed[-1][1] - timed[0][2]   # first start -> last end
        ev_ms = list(b["kernels_ms"].values())[0]
        summ["driver"] = {
            "command": "python3 bench.py --gpus 1 --steps 20 --warmup 5 (under rocprofv3 --kernel-trace --stats)",
            "kernel": b["roofline"]["kernel"], "timed_launches": len(timed), "stream_id": stream,
            "launches_on_stream": len(by[stream]),
            "avg_duration_us": round(avg_ns / 1e3, 2),
            "min_us": round(min(ns for _, ns, _ in timed) / 1e3, 2),
            "max_us": round(max(ns for _, ns, _ in timed) / 1e3, 2),
            "span_per_launch_us": round(span_ns / len(timed) / 1e3, 2),
            "alg_bytes_per_launch": alg,
            "achieved_GBs_from_trace": round(alg / avg_ns, 1),
            "frac_from_trace": round(alg / avg_ns / PEAK, 4),
            "bench_line_hip_event_ms": ev_ms, "bench_line_frac": b["roofline"]["frac"],
            "bench_line_value_GiBs": b["value"],
            "trace_vs_events": round(avg_ns / 1e6 / ev_ms, 4),
        }
        st = glob.glob(os.path.join(src, "driver", "**", "*kernel_stats.csv"), recursive=True)
        if st:
            shutil.copy(st[0], os.path.join(dst, "kernel_stats.csv"))
    # ---- PMC traffic
    tr = {}
    for name, ctr in (("fetch", "FETCH_SIZE"), ("write", "WRITE_SIZE")):
        sel = [r for r in rows(os.path.join(src, name, "**", "*counter_collection.csv"))
               if r.get("Counter_Name") == ctr and SMALL in r.get("Kernel_Name", "")]
        if not sel:
            continue
        with open(os.path.join(dst, f"pmc_{name}.csv"), "w", newline="") as fh:
            w = csv.DictWriter(fh, fieldnames=list(sel[0].keys()))
            w.writeheader()
            w.writerows(sel)
        vals = [float(r["Counter_Value"]) for r in sel]
        top = max(vals)
        full = [v for v in vals if v >= 0.9 * top]      # full-batch dispatches (not the count probe)
        tr[ctr] = sum(full[-3:]) / len(full[-3:]) * 1024.0
    if b and len(tr) == 2:
        alg = int(b["roofline"]["alg_bytes_per_launch"])
        hbm = 2.0 * tr["FETCH_SIZE"] + tr["WRITE_SIZE"]
        t = {"kernel": b["roofline"]["kernel"], "blocks": b["config"]["blocks_per_gpu"],
             "fetch_size_raw_bytes": tr["FETCH_SIZE"], "fetch_bytes_corrected": 2.0 * tr["FETCH_SIZE"],
             "write_bytes": tr["WRITE_SIZE"], "hbm_bytes_per_launch": hbm, "alg_bytes_per_launch": alg,
             "traffic_over_alg": round(hbm / alg, 4),
             "source": f"profiles/{RND}/{os.path.basename(dst)}/pmc_fetch.csv, pmc_write.csv "
                       "(rocprofv3 --pmc, separate passes, bench.py --steps 3 --warmup 1)",
             "note": "FETCH_SIZE x2 (gfx950 wide-read correction), KiB -> bytes; mean of the last 3 full-batch dispatches"}
        summ["traffic"] = t
        json.dump(t, open(os.path.join(ROOT, "profiles", "traffic.json"), "w"), indent=1)
    # ---- cfg2 at the cfg4 4 KiB leg's size, and the cfg4 legs
    b2 = bench_line(os.path.join(src, "cfg2_845k.log"))
    if b2:
        by = launches(os.path.join(src, "cfg2_845k"), SMALL)
        stream = max(by, key=lambda s: len(by[s]))
        timed = by[stream][-int(b2["steps"]):]
        avg = sum(ns for _, ns, _ in timed) / len(timed)
        summ["cfg2_845k"] = {"blocks": b2["config"]["blocks_per_gpu"], "value_GiBs": b2["value"],
                             "avg_launch_us": round(avg / 1e3, 1), "frac": b2["roofline"]["frac"],
                             "block_GiBs_from_trace": round(b2["config"]["block_bytes_per_gpu"] / avg * 1e9 / 2**30, 1)}
    b4 = bench_line(os.path.join(src, "cfg4_trace.log"))
    if b4:
        by = launches(os.path.join(src, "cfg4"), "")
        allr = sorted((x for v in by.values() for x in v))
        small = launches(os.path.join(src, "cfg4"), SMALL)
        large = launches(os.path.join(src, "cfg4"), LARGE)
        leg4 = b4["legs"].get("4096", {})
        s4 = max((v for v in small.values()), key=len) if small else []
        # the 4 KiB leg's launches are the biggest PipeSmall dispatches (16 KiB leg: fewer blocks)
        durs = sorted(ns for _, ns, _ in s4)
        summ["cfg4"] = {"value_GiBs": b4["value"], "legs": b4["legs"], "decode_launches": len(allr),
                        "pipe_small_launches": len(s4), "pipe_large_launches": sum(len(v) for v in large.values()),
                        "pipe_small_durations_us_quartiles": [round(durs[int(q * (len(durs) - 1))] / 1e3, 1)
                                                             for q in (0, 0.25, 0.5, 0.75, 1.0)] if durs else None,
                        "leg4_bytes": leg4.get("bytes")}
        st = glob.glob(os.path.join(src, "cfg4", "**", "*kernel_stats.csv"), recursive=True)
        if st:
            shutil.copy(st[0], os.path.join(dst, "cfg4_kernel_stats.csv"))
    json.dump(summ, open(os.path.join(dst, "summary.json"), "w"), indent=1)
    print(json.dumps(summ, indent=1))


if __name__ == "__main__":
    main()
