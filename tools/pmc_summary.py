#!/usr/bin/env python3
"""Summarise a rocprofv3 --pmc FETCH_SIZE pass (rocpd .db) for one kernel, per launch shape.

    python tools/pmc_summary.py <pmc run_results.db> [kernel-substring] [--latest LOG2N BATCH OUT.json]

FETCH_SIZE is in KiB per dispatch.  On gfx950 it reports HALF of the bytes of a wide
coalesced streaming read (16 B per lane; MI355X_MICROARCH.md, HBM section), so the HBM read
bytes are estimated as 2 * FETCH_SIZE * 1024; both numbers are written out.  The PMC pass
runs with --pmc only (no --sys-trace / --runtime-trace), its own process.

--latest writes the record bench.py reads for roofline.traffic (the launch shape with
grid_y == BATCH, i.e. BATCH MSMs of 2^LOG2N points per launch).
"""
import json
import os
import sqlite3
import sys
from collections import defaultdict

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def summarise(db, sub="msm_dlog_kernel"):
    c = sqlite3.connect(db)
    grid = {r[0]: (r[1], r[2], r[3], r[4]) for r in
            c.execute("select dispatch_id, grid_x, grid_y, workgroup_x, duration from kernels")}
    per = defaultdict(list)
    for name, did, cname, val in c.execute(
            "select name, dispatch_id, counter_name, counter_value from pmc_events"):
        if sub in name and "FETCH" in cname.upper():
            gx, gy, wx, _ = grid.get(did, (None, None, None, None))
            per[(name, gx, gy, wx)].append(float(val))
    out = []
    for (k, gx, gy, wx), vs in sorted(per.items(), key=lambda kv: -len(kv[1])):
        avg = sum(vs) / len(vs)
        out.append({"kernel": k, "grid": [gx, gy], "block": wx, "dispatches": len(vs),
                    "fetch_size_kib_avg": round(avg, 2),
                    "hbm_read_bytes_est": int(2 * avg * 1024)})
    return out


if __name__ == "__main__":
    args = sys.argv[1:]
    latest = None
    if "--latest" in args:
        i = args.index("--latest")
        latest = (int(args[i + 1]), int(args[i + 2]), args[i + 3])
        args = args[:i] + args[i + 4:]
    rows = summarise(args[0], *(args[1:2]))
    print(json.dumps(rows, indent=1))
    if latest:
        log2n, batch, path = latest
        match = [r for r in rows if r["grid"][1] == batch]
        if match:
            r = match[0]
            from bench import kernel_source_hash
            with open(path, "w") as f:
                json.dump({"log2n": log2n, "msm_batch": batch, "kernel": r["kernel"],
                           "source_sha16": kernel_source_hash(),
                           "grid": r["grid"], "block": r["block"], "dispatches": r["dispatches"],
                           "fetch_size_kib_avg": r["fetch_size_kib_avg"],
                           "hbm_bytes_per_launch": r["hbm_read_bytes_est"],
                           "alg_bytes_per_launch": 4 * (1 << log2n) * batch,
                           "method": "rocprofv3 --pmc FETCH_SIZE (own pass, bench.py --profile-only); "
                                     "HBM read bytes = 2 x FETCH_SIZE (gfx950 calibration, "
                                     "MI355X_MICROARCH.md HBM section)"}, f, indent=1)
