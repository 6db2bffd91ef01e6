#!/usr/bin/env python3
"""Summarise a tools/profile.sh run: per-kernel average duration (kernel trace) and HBM
bytes per launch from FETCH_SIZE / WRITE_SIZE (MI355X_MICROARCH.md: FETCH_SIZE counts half
the bytes of a 16-B/lane coalesced read -> x2; WRITE_SIZE exact for 16-B stores; units KB)."""
import csv
import glob
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
def argval(flag, default):
    toks = args.split()
    return int(toks[toks.index(flag) + 1]) if flag in toks else default


summary = {"tag": tag, "bench_args": args, "batch": argval("--batch", 256), "kp": argval("--kp", 1024),
           "kernels": {}}
for r in stats:
    name = r.get("Name", r.get("KernelName", "?"))
    short = short_name(name)
    summary["kernels"][short] = {"calls": int(r["Calls"]), "avg_ns": float(r["AverageNs"]),
                                 "total_ns": float(r["TotalDurationNs"]), "pct": float(r.get("Percentage", 0))}
for C in ("FETCH_SIZE", "WRITE_SIZE"):
    per = {}
    for r in rows("pmc_%s/**/*counter_collection.csv" % C):
        name = short_name(r.get("Kernel_Name", r.get("KernelName", "?")))
        if r.get("Counter_Name", C) != C:
            continue
        per.setdefault(name, []).append(float(r["Counter_Value"]))
    for k, v in per.items():
        summary["kernels"].setdefault(k, {})[C + "_KB_avg"] = sum(v) / len(v)
for k, v in summary["kernels"].items():
    if "FETCH_SIZE_KB_avg" in v or "WRITE_SIZE_KB_avg" in v:
        v["hbm_bytes_per_launch"] = 2 * v.get("FETCH_SIZE_KB_avg", 0) * 1024 + v.get("WRITE_SIZE_KB_avg", 0) * 1024
json.dump(summary, open(os.path.join(out, "summary_%s.json" % tag), "w"), indent=1)
print(json.dumps(summary, indent=1))
