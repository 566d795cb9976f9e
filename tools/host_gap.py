#!/usr/bin/env python3
"""Host-side HIP API calls of the LAST prove call in a rocprofv3 --hip-trace --kernel-trace run of
tools/prove_bench.py (tuning aid): every runtime call from the proof's first launch to the launch
of its first NTT pass, with its start offset and duration -- where the host spends the time that
shows up as a GPU gap between prep_kernel and the first forward pass.
    python tools/host_gap.py <run_results.db>"""
import sqlite3
import sys

db = sqlite3.connect(sys.argv[1])
names = [r[0] for r in db.execute("select name from sqlite_master where type in ('table', 'view')")]
if "regions" not in names:
    print("tables:", names)
    sys.exit(1)
cols = [r[1] for r in db.execute("pragma table_info(regions)")]
rows = list(db.execute("select name, start, end from regions order by start"))
kern = list(db.execute("select name, start, end from kernels order by start"))
# the last proof: its prep_kernel dispatch and the first wt_fwd after it
preps = [k for k in kern if "prep_kernel" in k[0]]
if not preps:
    print("no prep_kernel; columns", cols)
    sys.exit(1)
p = preps[-1]
fwd = next(k for k in kern if k[1] > p[1] and "wt_fwd_kernel" in k[0])
print("GPU: prep %.1f us, gap to first forward pass %.1f us" % ((p[2] - p[1]) / 1e3, (fwd[1] - p[2]) / 1e3))
# host calls from ~30 us before the prep dispatch starts to the forward pass's start
lo = p[1] - 60000
sel = [r for r in rows if lo <= r[1] <= fwd[1]]
t0 = sel[0][1] if sel else lo
for name, s, e in sel:
    print("%9.2f %8.2f  %s" % ((s - t0) / 1e3, (e - s) / 1e3, name[:80]))
print("prep dispatch start at %.2f, forward start at %.2f" % ((p[1] - t0) / 1e3, (fwd[1] - t0) / 1e3))
