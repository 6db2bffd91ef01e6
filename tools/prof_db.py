#!/usr/bin/env python3
"""Summarise a rocprofv3 results database (rocpd SQLite, the default output format): per kernel
(short name + grid) the dispatch count and mean duration; with --pmc the per-dispatch mean of
every collected counter (counters_collection view).  --json prints one JSON object instead."""
import json
import re
import sqlite3
import sys
from collections import defaultdict


def short(name):
    name = re.sub(r"^void ", "", name)
    name = name.replace("(anonymous namespace)::", "")
    m = re.match(r"([\w:]+(?:<[^()]*>)?)", name)
    return m.group(1) if m else name[:60]


def summarise(path):
    con = sqlite3.connect(path)
    cur = con.cursor()
    out = {}
    views = [r[0] for r in cur.execute("select name from sqlite_master where type in ('table','view')")]
    if "counters_collection" in views and cur.execute("select count(*) from counters_collection").fetchone()[0]:
        acc = defaultdict(lambda: defaultdict(list))
        for name, gs, dispatch, cn, v in cur.execute(
                "select kernel_name, grid_size, dispatch_id, counter_name, value from counters_collection"):
            acc[(short(name), gs)][cn].append(v)
        for (nm, gs), cs in acc.items():
            out["%s grid=%d" % (nm, gs)] = {c: sum(v) / len(v) for c, v in cs.items()}
        return out
    groups = defaultdict(list)
    for name, gx, gy, gz, du in cur.execute("select name, grid_x, grid_y, grid_z, duration from kernels order by start"):
        groups["%s grid=%d" % (short(name), gx * gy * gz)].append(du)
    for k, v in groups.items():
        out[k] = {"calls": len(v), "avg_us": sum(v) / len(v) / 1e3}
    return out


if __name__ == "__main__":
    s = summarise(sys.argv[1])
    if "--json" in sys.argv:
        print(json.dumps(s, indent=1))
    else:
        for k, v in s.items():
            print("%-70s %s" % (k[:70], " ".join("%s=%.4g" % kv for kv in v.items())))
