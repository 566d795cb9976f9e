#!/usr/bin/env python3
"""Per-kernel split of the LAST prove call in a rocprofv3 kernel trace of tools/prove_bench.py
(calls delimited by trim_pack_kernel or commit_pack_kernel, the last kernel of a proof).  python tools/prove_breakdown.py <run_results.db>"""
import collections
import sqlite3
import sys

rows = list(sqlite3.connect(sys.argv[1]).execute(
    "select name, duration, start, end from kernels order by start"))
idx = [i for i, r in enumerate(rows) if "trim_pack" in r[0] or "commit_pack" in r[0]]
seg = rows[idx[-2] + 1:idx[-1] + 1]
print("span_us %.1f kernels %d busy_us %.1f" % ((seg[-1][3] - seg[0][2]) / 1e3, len(seg),
                                               sum(r[1] for r in seg) / 1e3))
agg = collections.defaultdict(lambda: [0, 0.0])
for name, dur, _, _ in seg:
    k = name.replace("(anonymous namespace)::", "").split("(")[0][:64]
    agg[k][0] += 1
    agg[k][1] += dur / 1e3
for k, v in sorted(agg.items(), key=lambda kv: -kv[1][1]):
    print("%-64s %4d %9.1f" % (k, v[0], v[1]))
