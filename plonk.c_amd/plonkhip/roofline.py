"""Butterfly and byte accounting of NTT pass launches (records of plk_ntt_launch_log), shared by
bench.py (the C5 line's roofline) and tools/ntt_roofline.py (the rocprof recomputation), so both
price the same work against the same peaks.

Per launch record {kind, tb, m, k, n, per_block, units, field}: tiles = 2^k / 2^tb;
  forward / inverse pass (kind 0 / 1): n arrays x tiles x 2^(tb-1) x m radix-2 butterflies (the high
      passes' one column multiply per element not counted: a lower bound), 8 B per element per array
      (u32 read + write);
  centre (kind 2): tiles x units x 2^(tb-1) x tb (units = the lo = 0 passes it runs per tile: two
      forward transforms and one inverse per product, fixed operands' skipped passes excluded),
      12 B per element per product (two operands read, the product written);
  shared-operand lo = 0 pass (kind 3): n arrays x tiles x 2^(tb-1) x tb, 8 B per element per array.
Peaks: profiles/r02_bfly_peak.json (tools/bfly_peak.hip: the engine's own butterfly formulas in
registers at full occupancy) -- forward and shared passes DIF, inverse DIT, centre (2 DIF + 1 DIT) / 3."""
import json
import os

KINDS = {0: "fwd", 1: "inv", 2: "center", 3: "fix"}


def load_peaks(path):
    with open(path) as f:
        return json.loads([l for l in f if l.startswith("{")][0])


def peak_bfly_s(kind, field, pk):
    """butterflies per second of the roof for a launch of this kind (name or code) and field
    (0 / "F29", 1 / "FBB")"""
    kind = KINDS.get(kind, kind)
    f = "f29" if field in (0, "F29") else "bb"
    dif, dit = pk[f + "_dif_Gbfly_s"] * 1e9, pk[f + "_dit_Gbfly_s"] * 1e9
    if kind in ("fwd", "fix"):
        return dif
    if kind == "inv":
        return dit
    return 3.0 / (2.0 / dif + 1.0 / dit)


def launch_butterflies(r):
    tiles = (1 << r["k"]) >> r["tb"]
    half = 1 << (r["tb"] - 1)
    if r["kind"] == 2:
        return tiles * r["units"] * r["tb"] * half
    if r["kind"] == 3:
        return tiles * r["n"] * r["tb"] * half
    return tiles * r["n"] * r["m"] * half


def launch_bytes(r):
    elems = 1 << r["k"]
    return elems * r["n"] * (12 if r["kind"] == 2 else 8)


def plan_roofline(recs, pk):
    """totals over a list of launch records: butterflies, bytes, and the butterfly-roof time (s)"""
    bfly = sum(launch_butterflies(r) for r in recs)
    roof_s = sum(launch_butterflies(r) / peak_bfly_s(r["kind"], r.get("field", 0), pk) for r in recs)
    return {"butterflies": bfly, "bytes": sum(launch_bytes(r) for r in recs), "roof_s": roof_s,
            "launches": len(recs)}


PEAKS = os.path.join(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))), "profiles",
                     "r02_bfly_peak.json")
