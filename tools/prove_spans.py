#!/usr/bin/env python3
"""Kernel spans of every prove call in a rocprofv3 kernel trace of tools/prove_bench.py (calls
delimited by trim_pack_kernel / commit_pack_kernel; the first call dropped): min / median / max in us.
python tools/prove_spans.py <run_results.db>"""
import sqlite3
import sys

rows = list(sqlite3.connect(sys.argv[1]).execute("select name, start, end from kernels order by start"))
idx = [i for i, r in enumerate(rows) if "trim_pack" in r[0] or "commit_pack" in r[0]]
spans = sorted((rows[b][2] - rows[a + 1][1]) / 1e3 for a, b in zip(idx[1:-1], idx[2:]))
print("calls %d span_us min %.1f median %.1f max %.1f" % (len(spans), spans[0], spans[len(spans) // 2], spans[-1]))
