"""ORACLE -- test infrastructure only (tests/, __graft_entry__.smoke(), bench.py cpu_baseline).

CPU restatement of the reference prover, operation by operation:
  plonk_new            src/plonk.h:53-118   (h, cosets, inverse Vandermonde, Z_H)
  plonk_prove          src/plonk.h:223-656  (sigma, interpolation, rounds 1-5)
  poly_* helpers       src/poly.h:20-272    (trimming, add/sub/scale/add_hf, divide, eval, slice)
  srs_eval_at_s        src/srs.h:53-68      (degree check + serial fold)
with the heavy primitives (poly_mul, poly_divide, the MSM fold) delegated to the C oracle
(oracle.c).  Pinned against every proof -- and every rejected instance -- the compiled
reference produced in tests/golden/prove.json.  `rounds()` is the same code entered after the
interpolations, so prove-shaped runs at large n (synthetic polynomials, non-strict) have a
CPU answer to compare the device prover against.
"""
import numpy as np

P = 17
OMEGA, K1, K2 = 4, 2, 3   # src/plonk.h:12-14


class ProveError(Exception):
    """Where the reference calls exit() or fails an assert()."""


def _trim(c):
    c = np.asarray(c, dtype=np.uint8)
    n = c.size
    nz = np.flatnonzero(c)
    n = int(nz[-1]) + 1 if nz.size else min(n, 1)
    return c[:max(n, 1)].copy() if c.size else c.copy()


def hpow(b, e):
    return pow(int(b) % P, int(e), P)


def hinv(a):
    return pow(int(a) % P, P - 2, P)   # inv(0) = 0, as the hf_inverses LUT


def poly_add(a, b):
    n = max(len(a), len(b))
    out = np.zeros(n, np.int64)
    out[:len(a)] += a
    out[:len(b)] += b
    return _trim(out % P)


def poly_sub(a, b):
    n = max(len(a), len(b))
    out = np.zeros(n, np.int64)
    out[:len(a)] += a
    out[:len(b)] -= b
    return _trim(out % P)


def poly_scale(p, s):
    if s % P == 0:
        return np.zeros(1, np.uint8)
    return _trim(np.asarray(p, np.int64) * (s % P) % P)


def poly_add_hf(p, v):
    """Mutates p in place (src/poly.h:67-70) and returns it."""
    p[0] = (int(p[0]) + v) % P
    return p


def poly_eval(p, x):
    x %= P
    p = np.asarray(p, np.int64)
    if p.size == 0:
        return 0
    if x == 0:
        return int(p[0] % P)
    pw = np.array([pow(x, j, P) for j in range(16)], np.int64)
    return int((p * pw[np.arange(p.size) % 16]).sum() % P)


def poly_slice(p, start, end):
    if start >= end or end > len(p):
        raise ProveError("Invalid slice indices in poly_slice")
    return _trim(p[start:end])


class Prover:
    """plonk_prove restated; `orc` is an oracle.pyoracle.Oracle (C restatement)."""

    def __init__(self, orc, srs_g1, n, h=None, k1_h=None, k2_h=None, h_pows_inv=None, z_h=None):
        self.o = orc
        self.srs = np.frombuffer(bytes(srs_g1), np.uint8).reshape(-1, 3)
        self.n = n
        self.h = None if h is None else np.frombuffer(bytes(h), np.uint8)
        self.k1_h = None if k1_h is None else np.frombuffer(bytes(k1_h), np.uint8)
        self.k2_h = None if k2_h is None else np.frombuffer(bytes(k2_h), np.uint8)
        self.hinv = None if h_pows_inv is None else np.frombuffer(bytes(h_pows_inv), np.uint8).reshape(n, n)
        self.z_h = _trim(np.frombuffer(bytes(z_h), np.uint8))

    # -- heavy primitives -------------------------------------------------------------
    def mul(self, a, b):
        a, b = np.asarray(a, np.uint8), np.asarray(b, np.uint8)
        if min(len(a), len(b)) <= 64 or len(a) + len(b) < 4096:
            out = self.o.poly_mul(a, b)
        else:
            out = self.o.poly_mul_ntt(a, b)
        return _trim(np.frombuffer(out, np.uint8))

    def divide(self, num, den):
        q, r = self.o.poly_divide(num, den)
        return _trim(np.frombuffer(q, np.uint8)), _trim(np.frombuffer(r, np.uint8))

    def commit(self, p):
        if len(p) > len(self.srs):
            raise ProveError("SRS length is less than polynomial length")
        return self.o.msm(self.srs[:len(p)].reshape(-1), np.asarray(p, np.uint8))

    # -- src/plonk.h:162-195 --------------------------------------------------------------
    def interpolate(self, values):
        v = np.asarray(values, np.int64)
        return _trim(self.hinv.astype(np.int64) @ v % P)

    def prove(self, q_m, q_l, q_r, q_o, q_c, copies, a, b, c, chal, rnd):
        """copies: 3 lists of (type, index) pairs (type 0=A 1=B 2=C, index 1-based)."""
        n = self.n
        a, b, c = (np.asarray(x, np.int64) % P for x in (a, b, c))
        q_m, q_l, q_r, q_o, q_c = (np.asarray(x, np.int64) % P for x in (q_m, q_l, q_r, q_o, q_c))
        # assert(constraints_satisfy) src/constraints.h:145-171
        lhs = (q_l * a + q_r * b + q_o * c + q_m * (a * b % P) + q_c) % P
        bad = np.flatnonzero(lhs)
        if bad.size:
            raise ProveError("Constraint %d not satisfied." % bad[0])
        # copy_constraints_to_roots src/plonk.h:141-160
        roots = [self.h, self.k1_h, self.k2_h]
        sig = []
        for cp in copies:
            s = []
            for t, idx in cp:
                if t not in (0, 1, 2):
                    raise ProveError("Invalid copy_of type")
                s.append(int(roots[t][idx - 1]))
            sig.append(s)
        f = [self.interpolate(x) for x in (a, b, c, q_o, q_m, q_l, q_r, q_c, sig[0], sig[1], sig[2])]
        s1, s2, s3 = f[8], f[9], f[10]
        # round 2 grand product src/plonk.h:326-359
        al, be, ga = chal[0] % P, chal[1] % P, chal[2] % P
        acc = [1]
        for i in range(1, n):
            op = hpow(OMEGA, i - 1)
            den = (a[i - 1] + be * op + ga) * (b[i - 1] + be * (K1 * op % P) + ga) % P * \
                  (c[i - 1] + be * (K2 * op % P) + ga) % P
            e1, e2, e3 = poly_eval(s1, op), poly_eval(s2, op), poly_eval(s3, op)
            num = (a[i - 1] + be * e1 + ga) * (b[i - 1] + be * e2 + ga) % P * (c[i - 1] + be * e3 + ga) % P
            acc.append(int(acc[-1] * (den * hinv(num) % P) % P))
        acc_x = self.interpolate(acc)
        if poly_eval(acc_x, hpow(OMEGA, n)) != 1:
            raise ProveError("assertion acc_x(omega^n) == 1 failed")
        e0 = np.zeros(n, np.int64)
        e0[0] = 1
        l_1 = self.interpolate(e0)
        return self.rounds(f + [acc_x, l_1], chal, rnd, strict=True)

    # -- src/plonk.h:277-655 -----------------------------------------------------------------
    def rounds(self, polys, chal, rnd, strict=True):
        n = self.n
        fa, fb, fc, q_o, q_m, q_l, q_r, q_c, s1, s2, s3, acc_x, l_1 = [_trim(p) for p in polys]
        al, be, ga, z, v = (x % P for x in chal)
        b1, b2, b3, b4, b5, b6, b7, b8, b9 = (x % P for x in rnd)
        zh = self.z_h
        # round 1
        a_x = poly_add(self.mul(_trim([b2, b1]), zh), fa)
        b_x = poly_add(self.mul(_trim([b4, b3]), zh), fb)
        c_x = poly_add(self.mul(_trim([b6, b5]), zh), fc)
        a_s, b_s, c_s = self.commit(a_x), self.commit(b_x), self.commit(c_x)
        # round 2 (acc_x given)
        z_x = poly_add(self.mul(_trim([b9, b8, b7]), zh), acc_x)
        z_s = self.commit(z_x)
        # round 3
        t1 = poly_add(poly_add(self.mul(self.mul(a_x, b_x), q_m), self.mul(a_x, q_l)),
                      poly_add(self.mul(b_x, q_r), self.mul(c_x, q_o)))
        t1 = poly_add(poly_add(t1, np.zeros(1, np.uint8)), q_c)
        A2 = poly_scale(poly_add(a_x, _trim([ga, be])), al)
        B2 = poly_add(b_x, _trim([ga, be * K1 % P]))
        C2 = poly_add(c_x, _trim([ga, be * K2 % P]))
        t2 = self.mul(self.mul(self.mul(A2, B2), C2), z_x)
        A3 = poly_scale(poly_add_hf(poly_add(a_x, poly_scale(s1, be)), ga), al)
        B3 = poly_add_hf(poly_add(b_x, poly_scale(s2, be)), ga)
        C3 = poly_add_hf(poly_add(c_x, poly_scale(s3, be)), ga)
        zw = _trim(np.asarray(z_x, np.int64) * np.array([hpow(OMEGA, i) for i in range(len(z_x))], np.int64) % P)
        t3 = self.mul(self.mul(self.mul(A3, B3), C3), zw)
        t4 = self.mul(poly_scale(poly_add(z_x, _trim([P - 1])), hpow(al, 2)), l_1)
        num = poly_add(poly_sub(poly_add(t1, t2), t3), t4)
        t_x, rem = self.divide(num, zh)
        if strict and np.any(rem):
            raise ProveError("Non-zero remainder in t(x) division")
        part = n + 2
        t_lo = poly_slice(t_x, 0, part)
        t_mid = poly_slice(t_x, part, 2 * part)
        t_hi = poly_slice(t_x, 2 * part, len(t_x))
        t_lo_s, t_mid_s, t_hi_s = self.commit(t_lo), self.commit(t_mid), self.commit(t_hi)
        # round 4
        a_z, b_z, c_z = poly_eval(a_x, z), poly_eval(b_x, z), poly_eval(c_x, z)
        s1_z, s2_z = poly_eval(s1, z), poly_eval(s2, z)
        t_z, zw_z = poly_eval(t_x, z), poly_eval(zw, z)
        r1 = poly_add(poly_add(poly_add(poly_scale(q_m, a_z * b_z), poly_scale(q_l, a_z)),
                               poly_scale(q_r, b_z)), poly_scale(q_o, c_z))
        x1 = (a_z + be * z + ga) % P
        x2 = (b_z + be * K1 % P * z + ga) % P
        x3 = (c_z + be * K2 % P * z + ga) % P
        r2 = poly_scale(z_x, x1 * x2 % P * x3 % P * al)
        y1 = (a_z + be * s1_z + ga) % P
        y2 = (b_z + be * s2_z + ga) % P
        r3 = poly_scale(self.mul(z_x, poly_scale(s3, be * zw_z)), y1 * y2 % P * al)
        r4 = poly_scale(z_x, poly_eval(l_1, z) * hpow(al, 2))
        r_x = poly_add(poly_add(poly_add(r1, r2), r3), r4)
        r_z = poly_eval(r_x, z)
        # round 5 (poly_add_hf mutates its argument; a_x, r_x, z_x are not read afterwards)
        w = poly_add(poly_add(t_lo, poly_scale(t_mid, hpow(z, n + 2))), poly_scale(t_hi, hpow(z, 2 * n + 4)))
        w = poly_add_hf(w, (P - t_z) % P)
        w = poly_add(w, poly_scale(poly_add_hf(r_x.copy(), (P - r_z) % P), v))
        for k, (p, e) in enumerate(((a_x, a_z), (b_x, b_z), (c_x, c_z), (s1, s1_z), (s2, s2_z))):
            w = poly_add(w, poly_scale(poly_add_hf(p.copy(), (P - e) % P), hpow(v, k + 2)))
        w_q, rem1 = self.divide(w, _trim([(P - z) % P, 1]))
        if strict and np.any(rem1):
            raise ProveError("assertion poly_is_zero(&rem1) failed")
        zz = poly_add_hf(z_x.copy(), (P - zw_z) % P)
        w_o, rem2 = self.divide(zz, _trim([(P - z) * OMEGA % P, 1]))
        if strict and np.any(rem2):
            raise ProveError("assertion poly_is_zero(&rem2) failed")
        w_s, wo_s = self.commit(w_q), self.commit(w_o)
        proof = b"".join([a_s, b_s, c_s, z_s, t_lo_s, t_mid_s, t_hi_s, w_s, wo_s]) + \
            bytes([a_z, b_z, c_z, s1_z, s2_z, r_z, zw_z])
        return proof
