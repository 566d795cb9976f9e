#!/usr/bin/env python3
"""Per-kernel counter summary of the prover's NTT kernels (tools/ntt_pmc_r3.sh).

    python tools/ntt_pmc_summary.py A.db B.db C.db D.db

For every wt_* kernel shape (name, grid): average duration, VALU / LDS instruction counts, the
VALU-issue-bound time (SQ_INSTS_VALU wave-instructions x the measured 4.2 cycles per 32-bit
integer VALU wave-instruction at full occupancy, tools/isa_clock.hip, over 1024 SIMDs at
2.4 GHz) as a fraction of the duration, LDS bank-conflict cycles per LDS-array cycle, HBM
traffic (FETCH_SIZE x 2 per the gfx950 calibration + WRITE_SIZE, KiB -> bytes) against the
kernel's algorithmic bytes (8 B per element per pass: u32 read + write; byte-input / byte-output
passes 5 B), and VALU instructions per butterfly.  The SQ counters come from a subset of the
shader engines and are scaled by launched waves / SQ_WAVES.""" 
import json
import os
import re
import sqlite3
import sys
from collections import defaultdict

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "plonk.c_amd"))
from plonkhip import roofline as RL  # noqa: E402  (bench.py's launch accounting)

CLK = 2.4e9
SIMDS = 1024
CYC_PER_VALU = 4.2


def load(db):
    """per (kernel, grid, ordinal within one proof) averages; the ordinal separates launches of
    one kernel shape at different points of the proof (a proof starts with prep_kernel)"""
    c = sqlite3.connect(db)
    grid = {r[0]: (r[1], r[2], r[3], r[4]) for r in
            c.execute("select dispatch_id, grid_x, grid_y, workgroup_x, duration from kernels")}
    rows = list(c.execute("select dispatch_id, name, counter_name, counter_value from pmc_events order by dispatch_id"))
    names = {}
    for did, name, _, _ in rows:
        names[did] = name
    ordinal, seen = {}, defaultdict(int)
    for did in sorted(names):
        short = re.sub(r"^void ", "", names[did].replace("(anonymous namespace)::", "").split("(")[0])
        if "prep_kernel" in short:
            seen.clear()
        g = grid.get(did, (0, 0, 0, 0))
        ordinal[did] = (short, g[0], g[1], g[2], seen[(short, g[0], g[1])])
        seen[(short, g[0], g[1])] += 1
    acc = defaultdict(lambda: defaultdict(list))
    durs = defaultdict(dict)
    for did, name, cn, v in rows:
        if "wt_" not in name:
            continue
        key = ordinal[did]
        acc[key][cn].append(float(v))
        durs[key][did] = grid.get(did, (0, 0, 0, 0))[3]
    return acc, durs


def tile_bits(name):
    m = re.search(r"<(\d+), ?(\d+)(?:, ?(\d+))?", name)
    return (int(m.group(1)), int(m.group(2)), int(m.group(3)) if m.group(3) else None) if m else (None, None, None)


def load_plan():
    """--plan plan.json (tools/prove_plan.py): arrays per (kind, TB, M, tiles) of the proof's table
    passes -- their grid y counts array GROUPS since round 4 (several arrays per block) -- and the
    centre / shared-operand launch records in launch order (the persistent centre's grid says
    nothing about its items: its butterflies and bytes come from the record, plonkhip.roofline)"""
    if "--plan" not in sys.argv:
        return {}, {}
    with open(sys.argv[sys.argv.index("--plan") + 1]) as f:
        launches = json.load(f)["launches"]
    passes = {("fwd" if r["kind"] == 0 else "inv", r["tb"], r["m"], (1 << r["k"]) >> r["tb"]): r["n"]
              for r in launches if r["kind"] in (0, 1)}
    seq = defaultdict(list)
    for r in launches:
        if r["kind"] in (2, 3):
            seq["center" if r["kind"] == 2 else "fixfwd"].append(r)
    return passes, seq


def main():
    plan, seq = load_plan()
    dbs = [load(p) for p in sys.argv[1:5]]
    keys = set()
    for a, _ in dbs:
        keys |= set(a)
    print("%-50s %8s %9s %7s %7s %6s %8s %7s %7s" % ("kernel (blocks, y)#launch", "dur_us", "valu/bfly", "valu_t",
                                                   "ldsconf", "lds/va", "traffic", "alg_MB", "ratio"))
    print("  valu/bfly: VALU lane-instructions per radix-2 butterfly (column multiplies, loads, address math "
          "included); valu_t: VALU-issue-bound time / duration; ldsconf: bank-conflict cycles / LDS-array cycles; "
          "lds/va: LDS / VALU instructions; traffic: 2 x FETCH_SIZE + WRITE_SIZE; alg: 8 B (u32 in + out) or "
          "5 B (byte side) per element; wait: SQ_WAIT_ANY / SQ_WAVE_CYCLES")
    # launch order of the centre / shared-operand kernels within a proof (template arguments may differ
    # between the two batches, so order by first dispatch rather than by the name's ordinal)
    first = {}
    for key, ids in dbs[0][1].items():   # (one trace: dispatch ids of different runs do not compare)
        if ids:
            first[key] = min(ids)
    order = {}
    for kind in ("center", "fixfwd"):
        ks = sorted((k for k in first if ("wt_" + kind) in k[0] or (kind == "center" and "wt_center" in k[0])),
                    key=lambda k: first[k])
        for i, k in enumerate(ks):
            order[k] = i
    for key in sorted(keys, key=lambda k: (k[0], k[4])):
        name, gx, gy, wx, ordn = key
        cs = {}
        dur = []
        for a, d in dbs:
            for cn, v in a.get(key, {}).items():
                cs[cn] = sum(v) / len(v)
            dur += [x for x in d.get(key, {}).values() if x]
        if not dur:
            continue
        dus = sum(dur) / len(dur) / 1e3
        TB, R, M = tile_bits(name)
        blocks = gx // wx if wx else 0
        waves = blocks * gy * (wx // 64)
        # SQ counters are collected on a subset of the shader engines: scale by launched waves
        scale = waves / cs["SQ_WAVES"] if cs.get("SQ_WAVES") else None
        center = "center" in name
        bfly = None
        alg = None
        kseq = "center" if center else "fixfwd" if "fixfwd" in name else None
        if kseq and order.get(key, 99) < len(seq.get(kseq, [])):
            rec = seq[kseq][order[key]]
            bfly = RL.launch_butterflies(rec)
            alg = RL.launch_bytes(rec)
        elif TB and M is not None and not center and "fixfwd" not in name:
            kind = "fwd" if "wt_fwd" in name else "inv"
            arrays = plan.get((kind, TB, M, blocks), gy)   # (blocks of the x dimension = tiles)
            bfly = blocks * arrays * (1 << (TB - 1)) * M
            u8 = name.replace(" ", "").split(",")[3] == "true"
            alg = blocks * arrays * (1 << TB) * (5 if u8 else 8)
        valu = cs.get("SQ_INSTS_VALU", 0) * scale if scale else None
        vt = valu * CYC_PER_VALU / SIMDS / CLK * 1e6 if valu else None
        ldsc = cs.get("SQ_LDS_BANK_CONFLICT", 0) / cs["SQ_LDS_IDX_ACTIVE"] if cs.get("SQ_LDS_IDX_ACTIVE") else None
        fetch = cs.get("FETCH_SIZE")
        write = cs.get("WRITE_SIZE")
        traffic = (2 * fetch + write) * 1024 if fetch is not None and write is not None else None
        wait = cs.get("SQ_WAIT_ANY", 0) / cs["SQ_WAVE_CYCLES"] if cs.get("SQ_WAVE_CYCLES") else None
        print("%-50s %8.1f %9s %7s %7s %6s %8s %7s %7s  wait %s" % (
            ("%s (%d, %d)#%d" % (name[:40], blocks, gy, ordn)), dus,
            "%.2f" % (valu * 64 / bfly) if valu and bfly else "-",
            "%.2f" % (vt / dus) if vt else "-",
            "%.3f" % ldsc if ldsc is not None else "-",
            "%.2f" % (cs.get("SQ_INSTS_LDS", 0) / cs["SQ_INSTS_VALU"]) if cs.get("SQ_INSTS_VALU") else "-",
            "%.1fMB" % (traffic / 1e6) if traffic else "-",
            "%.1f" % (alg / 1e6) if alg else "-",
            "%.2f" % (traffic / alg) if traffic and alg else "-",
            "%.2f" % wait if wait is not None else "-"))
        print("    scale %.1f  " % (scale or 0) + " ".join("%s=%.4g" % (k, v) for k, v in sorted(cs.items())))


if __name__ == "__main__":
    main()
