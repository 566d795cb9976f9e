#!/usr/bin/env python3
"""Host-vs-GPU pacing of the LAST prove call in a rocprofv3 --kernel-trace --hip-runtime-trace
database of tools/prove_bench.py (tuning aid): for every kernel of the proof, when the host's launch
call ran and returned and when the kernel started -- slack = kernel start - launch return (near
the launch latency: the GPU waited for the host; large: the host was ahead) -- and every other HIP
call in the window.  A proof starts at prep_kernel (or scalars_init_kernel).
    python3 tools/prove_hostgap.py <run_results.db>"""
import sqlite3
import sys

db = sqlite3.connect(sys.argv[1])
ks = list(db.execute("select name, start, end, corr_id from kernels order by start"))
first = [i for i, r in enumerate(ks) if "prep_kernel" in r[0] or "scalars_init" in r[0]]
seg = ks[first[-1]:]
# the proof's HIP calls: from the previous proof's last kernel end (its synchronous call returns
# after it) to the end; the k-th kernel launch call among them launched the k-th kernel
regs = list(db.execute("select name, start, end from regions order by start"))
t_lo = ks[first[-1] - 1][2] if first[-1] > 0 else 0
win = [r for r in regs if r[1] >= t_lo]
launches = [r for r in win if "Launch" in r[0]]
t0 = seg[0][1]
print("times in us relative to the proof's first kernel start; api = the k-th launch call (start, duration)")
print("%-44s %9s %7s %9s %7s %8s" % ("kernel", "api_at", "api_us", "k_start", "k_us", "slack"))
for i, (name, s, e, c) in enumerate(seg):
    k = name.replace("(anonymous namespace)::", "").split("(")[0][:44]
    if i < len(launches):
        a = launches[i]
        print("%-44s %9.1f %7.1f %9.1f %7.1f %8.1f" % (k, (a[1] - t0) / 1e3, (a[2] - a[1]) / 1e3, (s - t0) / 1e3,
                                                     (e - s) / 1e3, (s - a[2]) / 1e3))
    else:
        print("%-44s %9s %7s %9.1f %7.1f" % (k, "-", "-", (s - t0) / 1e3, (e - s) / 1e3))
print("\nHIP calls after the previous proof's last kernel (us rel. to this proof's first kernel start):")
for name, s, e in win[:300]:
    print("%10.1f %8.1f  %s" % ((s - t0) / 1e3, (e - s) / 1e3, name[:70]))
print("last kernel end %.1f us; HIP calls in window: %d, launches %d, kernels %d" % (
    (seg[-1][2] - t0) / 1e3, len(win), len(launches), len(seg)))
