"""Seeded synthetic inputs shared by the golden-fixture script, the tests and bench.py.

Counter-based SplitMix64 (vectorised numpy, bit-stable across platforms):
    r_i = mix(seed + (i + 1) * 0x9E3779B97F4A7C15),  i = 0, 1, ...
Every stream is a pure function of (seed, n).
"""
import numpy as np

_GOLD = np.uint64(0x9E3779B97F4A7C15)
_M1 = np.uint64(0xBF58476D1CE4E5B9)
_M2 = np.uint64(0x94D049BB133111EB)

# kG for k = 0..16 on y^2 = x^3 + 3 over GF(101), G = (1, 2) (src/g1.h:22-24);
# pinned by tests/golden/g1.json (k = 0 is the identity {0, 0, 1}).
KG = [(0, 0, 1), (1, 2, 0), (68, 74, 0), (26, 45, 0), (65, 98, 0), (12, 32, 0), (32, 42, 0),
      (91, 35, 0), (18, 49, 0), (18, 52, 0), (91, 66, 0), (32, 59, 0), (12, 69, 0),
      (65, 3, 0), (26, 56, 0), (68, 27, 0), (1, 99, 0)]


def splitmix64(seed, n, offset=0):
    with np.errstate(over="ignore"):
        i = np.arange(offset + 1, offset + n + 1, dtype=np.uint64)
        z = np.uint64(seed) + i * _GOLD
        z = (z ^ (z >> np.uint64(30))) * _M1
        z = (z ^ (z >> np.uint64(27))) * _M2
        return z ^ (z >> np.uint64(31))


def all_points():
    """The 102 elements of E(F101) as canonical 3-byte encodings, identity first, then
    affine points in (x, y) order."""
    pts = [(0, 0, 1)]
    for x in range(101):
        rhs = (x * x * x + 3) % 101
        for y in range(101):
            if (y * y) % 101 == rhs:
                pts.append((x, y, 0))
    return np.array(pts, dtype=np.uint8)


def msm_inputs(seed, n, kind="subgroup"):
    """(points[n,3] uint8, scalars[n] uint8).

    kind = "subgroup": points kG, k uniform in [1,16]; scalars uniform in [0,16]
    kind = "full":     points uniform over all 102 group elements (identity and the
                       2-torsion point (48,0) included); scalars uniform in [0,16]
    kind = "bytes":    subgroup points; scalars uniform over all 256 byte values
                       (g1_mul takes the raw HF byte as a uint64 scalar, src/srs.h:63)
    """
    r = splitmix64(seed, 2 * n)
    rp, rs = r[:n], r[n:]
    if kind in ("subgroup", "bytes"):
        table = np.array(KG[1:], dtype=np.uint8)
        pts = table[(rp % np.uint64(16)).astype(np.int64)]
    elif kind == "full":
        table = all_points()
        pts = table[(rp % np.uint64(102)).astype(np.int64)]
    else:
        raise ValueError(kind)
    if kind == "bytes":
        sc = (rs & np.uint64(0xFF)).astype(np.uint8)
    else:
        sc = (rs % np.uint64(17)).astype(np.uint8)
    return np.ascontiguousarray(pts), np.ascontiguousarray(sc)


def poly_inputs(seed, la, lb, lead_nonzero=True, modulus=17):
    """Two coefficient vectors (uint8) with entries uniform in [0, modulus)."""
    r = splitmix64(seed, la + lb)
    a = (r[:la] % np.uint64(modulus)).astype(np.uint8)
    b = (r[la:] % np.uint64(modulus)).astype(np.uint8)
    if lead_nonzero:
        if la:
            a[-1] = 1 + a[-1] % 16
        if lb:
            b[-1] = 1 + b[-1] % 16
    return a, b


def digest(c):
    """SHA-256 of the raw bytes, hex -- the fixture digest for long outputs."""
    import hashlib
    return hashlib.sha256(np.asarray(c, dtype=np.uint8).tobytes()).hexdigest()


def prove_instance(n, seed, srs_len):
    """Prove-shaped synthetic instance (rounds 1-5 at n gates): 13 random 'interpolated'
    polynomials of length n, challenges / blinding scalars, Z_H = x^n - 1, an SRS over the whole
    group (tests/test_prove_gpu.py, tests/golden/make_prove_2_20.py, bench.py)."""
    r = splitmix64(seed, 13 * n + 64)
    polys = [(r[i * n:(i + 1) * n] % np.uint64(17)).astype(np.uint8) for i in range(13)]
    chal = [int(x % np.uint64(17)) for x in r[13 * n:13 * n + 5]]
    rnd = [int(x % np.uint64(17)) for x in r[13 * n + 5:13 * n + 14]]
    chal[3] = max(chal[3], 2)            # z: avoid the degenerate z in {0, 1}
    zh = np.zeros(n + 1, np.uint8)
    zh[0], zh[n] = 16, 1
    pts, _ = msm_inputs(seed ^ 0x5A5A, srs_len, "full")
    return polys, chal, rnd, zh, pts
