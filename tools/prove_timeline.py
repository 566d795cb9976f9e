#!/usr/bin/env python3
"""Ordered kernel timeline of the LAST prove call in a rocprofv3 kernel trace of
tools/prove_bench.py (tuning aid): offset, gap before, duration, grid, name.
    python tools/prove_timeline.py <run_results.db>"""
import sqlite3
import sys

rows = list(sqlite3.connect(sys.argv[1]).execute(
    "select name, duration, start, end, grid_x, grid_y, workgroup_x from kernels order by start"))
idx = [i for i, r in enumerate(rows) if "trim_pack" in r[0] or "commit_pack" in r[0]]
seg = rows[idx[-2] + 1:idx[-1] + 1]
t0, prev = seg[0][2], seg[0][2]
for name, dur, s, e, gx, gy, wx in seg:
    k = name.replace("(anonymous namespace)::", "").split("(")[0][:58]
    print("%8.1f %6.1f %7.1f  %8dx%-3d %-5d %s" % ((s - t0) / 1e3, (s - prev) / 1e3, dur / 1e3, gx // max(wx, 1), gy, wx, k))
    prev = e
