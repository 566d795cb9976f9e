#!/usr/bin/env python3
"""Summary of a tools/c3_pmc.sh counter run (config C3's kernels: the 2^20 F29 forward transform and
poly_mul 2^19 x 2^19): per kernel its traced duration and, from the per-SE counter averages (rocprofv3
reports each counter per shader engine: 32 SEs of 8 CUs on MI355X), the VALU issue share of the SE's
busy time (VALU wave-instructions per SIMD x 4.2 cycles, the measured integer issue interval at full
occupancy, tools/isa_clock.hip), the waves' wait share, VALU per wave, LDS bank-conflict share and
fetched / written bytes.
    python tools/c3_pmc_summary.py <c3_pmc dir> [label]"""
import os
import re
import sys

d = sys.argv[1]
label = sys.argv[2] if len(sys.argv) > 2 else d


def rows(fn):
    out = {}
    for line in open(os.path.join(d, fn)):
        m = re.match(r"(.+?)\s+grid=\((\d+), (\d+)\) n=(\d+) (.*)", line.strip())
        if not m:
            continue
        vals = dict((k, float(v)) for k, v in (kv.split("=") for kv in m.group(5).split()))
        out.setdefault((m.group(1).strip(), int(m.group(2)), int(m.group(3))), {}).update(vals)
    return out


cnt = {}
for f in ("A.txt", "B.txt", "C.txt", "D.txt"):
    for k, v in rows(f).items():
        cnt.setdefault(k, {}).update(v)
def norm(name):   # the trace's names carry "(anonymous namespace)::" and are cut at 60 characters
    return name.replace("(anonymous namespace)::", "")[:30]


dur = {}
for line in open(os.path.join(d, "durations.txt")):
    m = re.match(r"(.+?)\s+grid=(\d+)x(\d+)\s+blk=(\d+)\s+calls=(\d+)\s+avg=\s*([\d.]+) us\s+med=\s*([\d.]+)", line.strip())
    if m:
        dur[(int(m.group(2)), int(m.group(3)), norm(m.group(1)))] = (float(m.group(6)), float(m.group(7)), int(m.group(4)))
print("# C3 counter pass (%s): per-SE averages, 32 SEs x 8 CUs x 4 SIMDs" % label)
print("%-44s %10s %7s %7s %9s %9s %8s %9s %9s %9s" % ("kernel", "grid", "avg_us", "w/SIMD", "VALU/wave", "VALUissue",
                                                  "wait", "LDSconfl", "fetch_MB", "write_MB"))
for (name, gx, gy), c in sorted(cnt.items(), key=lambda kv: -kv[1].get("SQ_BUSY_CYCLES", 0)):
    key = next((k for k in dur if k[0] == gx and k[1] == gy and (norm(name) == k[2] or k[2].startswith(norm(name) + "("))), None)
    avg, med, blk = dur[key] if key else (float("nan"), float("nan"), 0)
    waves = c.get("SQ_WAVES", 0)
    valu = c.get("SQ_INSTS_VALU", c.get("SQ_ACTIVE_INST_VALU", 0))
    issue = valu / 32.0 * 4.2 / c["SQ_BUSY_CYCLES"] if c.get("SQ_BUSY_CYCLES") else float("nan")
    wait = c.get("SQ_WAIT_ANY", 0) / c["SQ_WAVE_CYCLES"] if c.get("SQ_WAVE_CYCLES") else float("nan")
    lds = c.get("SQ_LDS_BANK_CONFLICT", 0) / c["SQ_LDS_IDX_ACTIVE"] if c.get("SQ_LDS_IDX_ACTIVE") else float("nan")
    wps = waves / 32.0   # (a launch's waves per SE over its 32 SIMDs: all resident at once in these launches)
    print("%-44s %10s %7.2f %7.1f %9.0f %9.2f %8.2f %9.3f %9.2f %9.2f" % (
        name[:44], "%dx%d" % (gx, gy), avg, wps, valu / waves if waves else 0, issue, wait, lds,
        2 * c.get("FETCH_SIZE", 0) * 1024 / 1e6, c.get("WRITE_SIZE", 0) * 1024 / 1e6))
print("VALUissue = SQ_INSTS_VALU / 32 SIMDs x 4.2 cycles / SQ_BUSY_CYCLES; wait = SQ_WAIT_ANY / SQ_WAVE_CYCLES; "
      "LDSconfl = SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE; fetch_MB = 2 x FETCH_SIZE (KiB per launch, the gfx950 calibration), write_MB = WRITE_SIZE")
