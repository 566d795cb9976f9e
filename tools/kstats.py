#!/usr/bin/env python3
"""Summarise a rocprofv3 kernel trace (rocpd SQLite .db, ROCm 7.2 default output):
per kernel (name, grid) -> calls, avg / median / min duration in microseconds.

    python tools/kstats.py gpurun_out/prof/run_results.db [name-substring] [--json out.json]
"""
import json
import sqlite3
import sys
from collections import defaultdict


def kernel_rows(db, sub=None):
    c = sqlite3.connect(db)
    q = "select name, grid_x, grid_y, workgroup_x, duration from kernels"
    out = defaultdict(list)
    for name, gx, gy, wx, dur in c.execute(q):
        if sub and sub not in name:
            continue
        out[(name, gx, gy, wx)].append(dur / 1000.0)
    return out


def summarise(db, sub=None):
    res = []
    for (name, gx, gy, wx), ds in sorted(kernel_rows(db, sub).items(), key=lambda kv: -sum(kv[1])):
        ds.sort()
        res.append({"kernel": name, "grid": [gx, gy], "block": wx, "calls": len(ds),
                    "avg_us": round(sum(ds) / len(ds), 3), "median_us": round(ds[len(ds) // 2], 3),
                    "min_us": round(ds[0], 3), "total_us": round(sum(ds), 1)})
    return res


if __name__ == "__main__":
    width = 60
    if "--wide" in sys.argv:
        width = 110
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    out_json = None
    if "--json" in sys.argv:
        out_json = sys.argv[sys.argv.index("--json") + 1]
        args = [a for a in args if a != out_json]
    db = args[0]
    sub = args[1] if len(args) > 1 else None
    rows = summarise(db, sub)
    for r in rows:
        print("%-*s grid=%-14s blk=%-5d calls=%-6d avg=%9.3f us  med=%9.3f  min=%9.3f" % (
            width, r["kernel"][:width], "%dx%d" % tuple(r["grid"]), r["block"], r["calls"], r["avg_us"],
            r["median_us"], r["min_us"]))
    if out_json:
        with open(out_json, "w") as f:
            json.dump(rows, f, indent=1)
