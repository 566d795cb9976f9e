#!/usr/bin/env python3
"""Per-kernel averages of every PMC counter in a rocprofv3 --pmc database (tuning aid).
    python tools/pmc_kernels.py run_results.db [name-substring]"""
import sqlite3
import sys
from collections import defaultdict

db = sys.argv[1]
sub = sys.argv[2] if len(sys.argv) > 2 else ""
c = sqlite3.connect(db)
grid = {r[0]: (r[1], r[2]) for r in c.execute("select dispatch_id, grid_x, grid_y from kernels")}
acc = defaultdict(lambda: defaultdict(list))
for name, did, cn, v in c.execute("select name, dispatch_id, counter_name, counter_value from pmc_events"):
    if sub in name:
        k = (name.replace("(anonymous namespace)::", "").split("(")[0][:60], grid.get(did))
        acc[k][cn].append(v)
for (name, g), cs in sorted(acc.items()):
    vals = " ".join("%s=%.4g" % (cn, sum(v) / len(v)) for cn, v in sorted(cs.items()))
    print("%-60s grid=%s n=%d %s" % (name, g, len(next(iter(cs.values()))), vals))
