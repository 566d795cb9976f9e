#!/usr/bin/env python3
"""Compute roofline of the NTT kernels: butterflies per launch / duration / the measured
butterfly peak (tools/bfly_peak.hip: the engine's own butterfly formulas in registers, no memory,
full occupancy -- the integer-VALU roof of this arithmetic on this chip).

    python tools/ntt_roofline.py <run_results.db> <bfly_peak.json> [--prove [--plan plan.json] | --all] [--json out]

--prove: the kernels of the LAST prove call of the trace (tools/prove_bench.py; calls end with
trim_pack_kernel or commit_pack_kernel); --all (default): every wt_* dispatch, aggregated per (kernel, grid).

Butterflies counted (the algorithmic work, radix-2 count):
  wt_fwd/wt_inv_kernel<TB, R, M, ...>: blocks x 2^(TB-1) x M  (blocks = grid_x / workgroup x grid_y;
      the high passes' one column multiply per element is NOT counted, so the fraction is a lower
      bound; sum-group members have no inverse blocks)
  wt_center_kernel<TB, R, F>: (job, tile) items x 2^(TB-1) x TB x 3 (two forward transforms and one
      inverse per item); the items are the next inverse pass's blocks (same batch).  An estimate:
      fixed operands' skipped passes are counted, merged sum-group members' forward passes are
      not (the prover's 2^21 batch: 24 counted per tile for 22 run; 2^22: 6 for 8)
Peak: F29 / BabyBear DIF for forward passes, DIT for inverse, (2 DIF + 1 DIT) / 3 for the center.

--plan (tools/prove_plan.py, round 4): the proof's launch plan from the library
(plk_ntt_launch_log), matched to the pass kernels of the last proof in launch order.  Table passes
now walk several arrays per block (grid y = array groups, not arrays), and the plan gives the
exact counts: arrays x tiles x 2^(TB-1) x M for a pass, tiles x pass units x 2^(TB-1) x TB for the
center (the lo = 0 passes it actually runs, fixed operands' skipped passes excluded)."""
import json
import os
import re
import sqlite3
import sys
from collections import defaultdict

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "plonk.c_amd"))
from plonkhip import roofline as RL  # noqa: E402  (the same accounting as bench.py's C5 line)

PAT = re.compile(r"wt_(fwd|inv|center|fixfwd)_kernel<(\d+), (\d+)(?:, (\d+))?.*?(F29|FBB)")
KIND = {"fwd": 0, "inv": 1, "center": 2, "fixfwd": 3}


def parse(name):
    m = PAT.search(name.replace("(anonymous namespace)::", ""))
    if not m:
        return None
    kind, tb, _r, mm, field = m.groups()
    return kind, int(tb), int(mm) if mm else int(tb), field


def peak(kind, field, pk):
    return RL.peak_bfly_s(KIND[kind], field, pk)


def main():
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    db, pk_path = args[0], args[1]
    out_json = sys.argv[sys.argv.index("--json") + 1] if "--json" in sys.argv else None
    with open(pk_path) as f:
        pk = json.loads([l for l in f if l.startswith("{")][0])
    rows = list(sqlite3.connect(db).execute(
        "select name, grid_x, grid_y, workgroup_x, duration, start from kernels order by start"))
    if "--prove" in sys.argv:
        idx = [i for i, r in enumerate(rows) if "trim_pack" in r[0] or "commit_pack" in r[0]]
        rows = rows[idx[-2] + 1:idx[-1] + 1]
    # (--all --plan: the plan of the whole traced run, every pass launch in order)
    plan = None
    if "--plan" in sys.argv:
        with open(sys.argv[sys.argv.index("--plan") + 1]) as f:
            plan = [r for r in json.load(f)["launches"] if r["kind"] in (0, 1, 2, 3)]
    disp = []
    pi = 0
    for i, (name, gx, gy, wx, dur, _) in enumerate(rows):
        p = parse(name)
        if not p:
            continue
        kind, tb, mm, field = p
        if plan is not None:
            r = plan[pi]
            pi += 1
            if r["kind"] != KIND[kind] or r["tb"] != tb or r["m"] != mm:
                raise SystemExit("plan mismatch at %s: %r" % (name, r))
            bfly = RL.launch_butterflies(r)
            disp.append((name.replace("(anonymous namespace)::", "").split("(")[0], gx, gy, kind, field, bfly, dur / 1e3))
            continue
        if kind == "fixfwd":
            bfly = (gx // wx) * gy * (1 << (tb - 1)) * tb
        elif kind == "center":
            nxt = next((r for r in rows[i + 1:] if parse(r[0]) and parse(r[0])[0] == "inv"), None)
            if nxt is None:
                continue
            items = (nxt[1] // nxt[3]) * nxt[2]
            bfly = items * (1 << (tb - 1)) * tb * 3
        else:
            bfly = (gx // wx) * gy * (1 << (tb - 1)) * mm
        disp.append((name.replace("(anonymous namespace)::", "").split("(")[0], gx, gy, kind, field, bfly, dur / 1e3))
    agg = defaultdict(lambda: [0, 0, 0.0, None, None])
    for name, gx, gy, kind, field, bfly, us in disp:
        a = agg[(name, gx, gy)]
        a[0] += 1
        a[1] += bfly
        a[2] += us
        a[3], a[4] = kind, field
    res = []
    print("# butterfly roofline (peak: %s)" % pk_path)
    print("%-58s %-14s %5s %10s %12s %10s %6s" % ("kernel", "grid", "calls", "avg_us", "Mbfly/launch", "Gbfly/s", "frac"))
    tot_b = tot_t = tot_peak_t = 0.0
    for (name, gx, gy), (calls, bfly, us, kind, field) in sorted(agg.items(), key=lambda kv: -kv[1][2]):
        rate = bfly / (us * 1e-6)
        pkr = peak(kind, field, pk)
        frac = rate / pkr
        tot_b += bfly
        tot_t += us
        tot_peak_t += bfly / pkr * 1e6
        res.append({"kernel": name, "grid": [gx, gy], "calls": calls, "avg_us": round(us / calls, 2),
                    "bfly_per_launch": bfly // calls, "Gbfly_s": round(rate / 1e9, 1),
                    "peak_Gbfly_s": round(pkr / 1e9, 1), "frac": round(frac, 3)})
        print("%-58s %-14s %5d %10.2f %12.2f %10.1f %6.3f" % (name[:58], "(%d,%d)" % (gx, gy), calls, us / calls,
                                                          bfly / calls / 1e6, rate / 1e9, frac))
    if tot_t:
        print("all NTT kernels: %.1f us, butterfly-roof time %.1f us -> frac %.3f" % (tot_t, tot_peak_t,
                                                                                  tot_peak_t / tot_t))
    if out_json:
        with open(out_json, "w") as f:
            json.dump({"peak": pk, "kernels": res, "total_us": round(tot_t, 1),
                       "roof_us": round(tot_peak_t, 1), "frac": round(tot_peak_t / tot_t, 3) if tot_t else None},
                      f, indent=1)


if __name__ == "__main__":
    main()
