#!/usr/bin/env python3
"""Summarise a tools/profile.sh run: per-kernel average duration (kernel trace) and HBM
bytes per launch from FETCH_SIZE / WRITE_SIZE (MI355X_MICROARCH.md: FETCH_SIZE counts half
the bytes of a 16-B/lane coalesced read -> x2; WRITE_SIZE exact for 16-B stores; units KB)."""
import csv
import glob
import re
import json
import os
import sys

out, tag, args = sys.argv[1], sys.argv[2], sys.argv[3] if len(sys.argv) > 3 else ""


def short_name(name):
    name = name.replace("(anonymous namespace)::", "")
    if name.startswith("void "):
        name = name[5:]
    return name.split("(")[0].split("<")[0].split("::")[-1].strip()


def rows(pattern):
    res = []
    for f in glob.glob(os.path.join(out, pattern), recursive=True):
        with open(f) as fh:
            res += list(csv.DictReader(fh))
    return res


stats = rows("trace/**/*kernel_stats.csv")
def bench_default(flag):
    """bench.py's own argparse default for `flag` (the profile ran bench.py with these)."""
    src = open(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "bench.py")).read()
    m = re.search(r'add_argument\("%s", type=int, default=(\d+)' % re.escape(flag), src)
    return int(m.group(1))


def argval(flag):
    toks = args.split()
    return int(toks[toks.index(flag) + 1]) if flag in toks else bench_default(flag)


summary = {"tag": tag, "bench_args": args, "batch": argval("--batch"), "kp": argval("--kp"),
           "kernels": {}}
for r in stats:
    name = r.get("Name", r.get("KernelName", "?"))
    short = short_name(name)
    summary["kernels"][short] = {"calls": int(r["Calls"]), "avg_ns": float(r["AverageNs"]),
                                 "total_ns": float(r["TotalDurationNs"]), "pct": float(r.get("Percentage", 0))}
# median launch duration from the trace (the mean carries the first, cold launch)
durs = {}
for r in rows("trace/**/*kernel_trace.csv"):
    durs.setdefault(short_name(r.get("Kernel_Name", "?")), []).append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
for k, v in durs.items():
    if k in summary["kernels"]:
        v = sorted(v)
        summary["kernels"][k]["median_ns"] = float(v[len(v) // 2] if len(v) % 2 else (v[len(v) // 2 - 1] + v[len(v) // 2]) / 2)
per = {}
for r in rows("pmc_*/**/*counter_collection.csv"):
    name = short_name(r.get("Kernel_Name", r.get("KernelName", "?")))
    per.setdefault((name, r["Counter_Name"]), []).append(float(r["Counter_Value"]))
for (k, c), v in per.items():
    key = c + "_KB_avg" if c in ("FETCH_SIZE", "WRITE_SIZE") else c + "_avg"
    summary["kernels"].setdefault(k, {})[key] = sum(v) / len(v)
for k, v in summary["kernels"].items():
    if "FETCH_SIZE_KB_avg" in v or "WRITE_SIZE_KB_avg" in v:
        v["hbm_bytes_per_launch"] = 2 * v.get("FETCH_SIZE_KB_avg", 0) * 1024 + v.get("WRITE_SIZE_KB_avg", 0) * 1024
for k, v in summary["kernels"].items():
    if "GRBM_GUI_ACTIVE_avg" in v and "avg_ns" in v:
        v["effective_clock_GHz"] = v["GRBM_GUI_ACTIVE_avg"] / 8 / v["avg_ns"]
    if "SQ_VALU_MFMA_BUSY_CYCLES_avg" in v and "GRBM_GUI_ACTIVE_avg" in v:
        # MFMA busy cycles summed over SIMDs (1024) vs GPU-active cycles (summed over 8 XCDs)
        v["mfma_busy_frac"] = v["SQ_VALU_MFMA_BUSY_CYCLES_avg"] / (1024 * v["GRBM_GUI_ACTIVE_avg"] / 8)
json.dump(summary, open(os.path.join(out, "summary_%s.json" % tag), "w"), indent=1)
print(json.dumps(summary, indent=1))
