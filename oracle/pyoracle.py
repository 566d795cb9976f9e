"""ORACLE -- test infrastructure only (tests/, __graft_entry__.smoke(), bench.py cpu_baseline).

ctypes wrappers over
  * oracle/liboracle.so        -- our CPU restatement of the reference hot path (oracle.c)
  * oracle/_ref/libplonkref.so -- the unmodified reference headers compiled in place
                                  (ref_harness.c); absent on machines that never had
                                  /root/reference and no prebuilt copy.
Everything is plain bytes: a G1 is 3 bytes {x, y, infinite}, an HF is 1 byte.
"""
import ctypes as C
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
_u8p = C.POINTER(C.c_uint8)


def _ptr(a):
    return a.ctypes.data_as(_u8p)


def _u8(a):
    if isinstance(a, (bytes, bytearray)):
        return np.frombuffer(bytes(a), dtype=np.uint8).copy()
    return np.ascontiguousarray(np.asarray(a, dtype=np.uint8))


class _Lib:
    def __init__(self, path, prefix):
        self.path = path
        self.lib = C.CDLL(path)
        self.p = prefix
        L = self.lib
        for name, res, args in [
            ("g1_add", None, [_u8p, _u8p, _u8p]),
            ("g1_double", None, [_u8p, _u8p]),
            ("g1_mul", None, [_u8p, C.c_uint64, _u8p]),
            ("g1_is_on_curve", C.c_int, [_u8p]),
            ("msm" if prefix == "ref_" else "msm_fold", None, [_u8p, _u8p, C.c_size_t, _u8p]),
            ("poly_mul", C.c_size_t, [_u8p, C.c_size_t, _u8p, C.c_size_t, _u8p]),
            ("poly_eval", C.c_uint8, [_u8p, C.c_size_t, C.c_uint8]),
            ("matrix_mul", None, [_u8p, C.c_size_t, C.c_size_t, _u8p, C.c_size_t, _u8p]),
            ("matrix_inv", None, [_u8p, C.c_size_t, _u8p]),
        ]:
            f = getattr(L, prefix + name)
            f.restype = res
            f.argtypes = args

    def fn(self, name):
        return getattr(self.lib, self.p + name)

    def matrix_mul(self, a, m, k, b, n):
        a, b = _u8(a), _u8(b)
        out = np.zeros(max(m * n, 1), np.uint8)
        self.fn("matrix_mul")(_ptr(a), m, k, _ptr(b), n, _ptr(out))
        return bytes(out[:m * n])

    def matrix_inv(self, a, n):
        a = _u8(a)
        out = np.zeros(max(n * n, 1), np.uint8)
        self.fn("matrix_inv")(_ptr(a), n, _ptr(out))
        return bytes(out[:n * n])

    def g1_add(self, a, b):
        out = np.zeros(3, np.uint8)
        self.fn("g1_add")(_ptr(_u8(a)), _ptr(_u8(b)), _ptr(out))
        return bytes(out)

    def g1_double(self, a):
        out = np.zeros(3, np.uint8)
        self.fn("g1_double")(_ptr(_u8(a)), _ptr(out))
        return bytes(out)

    def g1_mul(self, a, k):
        out = np.zeros(3, np.uint8)
        self.fn("g1_mul")(_ptr(_u8(a)), int(k), _ptr(out))
        return bytes(out)

    def g1_is_on_curve(self, a):
        return bool(self.fn("g1_is_on_curve")(_ptr(_u8(a))))

    def poly_mul(self, a, b):
        a, b = _u8(a), _u8(b)
        out = np.zeros(max(len(a) + len(b) - 1, 1), np.uint8)
        n = self.fn("poly_mul")(_ptr(a), len(a), _ptr(b), len(b), _ptr(out))
        return bytes(out[:n])

    def poly_eval(self, p, x):
        p = _u8(p)
        return int(self.fn("poly_eval")(_ptr(p), len(p), int(x)))


class Oracle(_Lib):
    """Our restatement (oracle.c)."""

    def __init__(self, path=os.path.join(HERE, "liboracle.so")):
        super().__init__(path, "orc_")
        L = self.lib
        L.orc_msm_dlog.restype = C.c_int
        L.orc_msm_dlog.argtypes = [_u8p, _u8p, C.c_size_t, _u8p]
        L.orc_dlog.restype = C.c_int
        L.orc_dlog.argtypes = [_u8p]
        L.orc_dlog_exp.argtypes = [C.c_int, _u8p]
        L.orc_dlog_generator.argtypes = [_u8p]
        L.orc_poly_mul_ntt.restype = C.c_size_t
        L.orc_poly_mul_ntt.argtypes = [_u8p, C.c_size_t, _u8p, C.c_size_t, _u8p]
        L.orc_poly_mul_ntt_blocked.restype = C.c_size_t
        L.orc_poly_mul_ntt_blocked.argtypes = [_u8p, C.c_size_t, _u8p, C.c_size_t, _u8p, C.c_size_t]
        L.orc_poly_divide.restype = C.c_int
        L.orc_poly_divide.argtypes = [_u8p, C.c_size_t, _u8p, C.c_size_t, _u8p,
                                      C.POINTER(C.c_size_t), _u8p, C.POINTER(C.c_size_t)]
        L.orc_gen_survey_msm.argtypes = [C.c_size_t, _u8p, _u8p]
        L.orc_gen_survey_poly.argtypes = [C.c_size_t, _u8p, _u8p]
        L.orc_digest31.restype = C.c_uint32
        L.orc_digest31.argtypes = [_u8p, C.c_size_t]

    def msm(self, pts, sc):
        """Serial fold exactly as srs_eval_at_s."""
        pts, sc = _u8(pts).reshape(-1), _u8(sc)
        assert pts.size == 3 * sc.size
        out = np.zeros(3, np.uint8)
        self.lib.orc_msm_fold(_ptr(pts), _ptr(sc), sc.size, _ptr(out))
        return bytes(out)

    def msm_dlog(self, pts, sc):
        """(log, G1 bytes) for canonical on-curve inputs; (None, None) if irregular."""
        pts, sc = _u8(pts).reshape(-1), _u8(sc)
        out = np.zeros(3, np.uint8)
        r = self.lib.orc_msm_dlog(_ptr(pts), _ptr(sc), sc.size, _ptr(out))
        return (None, None) if r < 0 else (r, bytes(out))

    def dlog(self, p):
        r = self.lib.orc_dlog(_ptr(_u8(p)))
        return None if r < 0 else r

    def dlog_exp(self, k):
        out = np.zeros(3, np.uint8)
        self.lib.orc_dlog_exp(int(k), _ptr(out))
        return bytes(out)

    def dlog_generator(self):
        out = np.zeros(3, np.uint8)
        self.lib.orc_dlog_generator(_ptr(out))
        return bytes(out)

    def poly_mul_ntt(self, a, b):
        a, b = _u8(a), _u8(b)
        out = np.zeros(len(a) + len(b) - 1, np.uint8)
        n = self.lib.orc_poly_mul_ntt(_ptr(a), len(a), _ptr(b), len(b), _ptr(out))
        if n == 0:
            raise ValueError("orc_poly_mul_ntt: size out of range")
        return bytes(out[:n])

    def poly_mul_ntt_blocked(self, a, b, piece):
        """orc_poly_mul_ntt_blocked: the shorter operand in pieces of at most `piece` coefficients"""
        a, b = _u8(a), _u8(b)
        out = np.zeros(len(a) + len(b) - 1, np.uint8)
        n = self.lib.orc_poly_mul_ntt_blocked(_ptr(a), len(a), _ptr(b), len(b), _ptr(out), int(piece))
        if n == 0:
            raise ValueError("orc_poly_mul_ntt_blocked: bad arguments")
        return bytes(out[:n])

    def poly_divide(self, num, den):
        num, den = _u8(num), _u8(den)
        q = np.zeros(max(len(num), 1), np.uint8)
        r = np.zeros(max(len(num), 1), np.uint8)
        lq, lr = C.c_size_t(), C.c_size_t()
        rc = self.lib.orc_poly_divide(_ptr(num), len(num), _ptr(den), len(den), _ptr(q),
                                      C.byref(lq), _ptr(r), C.byref(lr))
        if rc != 0:
            raise ZeroDivisionError("division by zero polynomial")
        return bytes(q[:lq.value]), bytes(r[:lr.value])

    def gen_survey_msm(self, n):
        pts = np.zeros(3 * n, np.uint8)
        sc = np.zeros(n, np.uint8)
        self.lib.orc_gen_survey_msm(n, _ptr(pts), _ptr(sc))
        return pts, sc

    def gen_survey_poly(self, n):
        a = np.zeros(n, np.uint8)
        b = np.zeros(n, np.uint8)
        self.lib.orc_gen_survey_poly(n, _ptr(a), _ptr(b))
        return a, b

    def digest31(self, c):
        c = _u8(c)
        return int(self.lib.orc_digest31(_ptr(c), c.size))


class Reference(_Lib):
    """The compiled reference headers (ref_harness.c) -- only where oracle/_ref exists."""

    def __init__(self, path=os.path.join(HERE, "_ref", "libplonkref.so")):
        super().__init__(path, "ref_")
        L = self.lib
        L.ref_prove4.restype = C.c_int
        L.ref_prove4.argtypes = [_u8p, _u8p, _u8p, _u8p, _u8p, C.c_uint8, C.c_size_t,
                                 C.c_int, _u8p]
        L.ref_interpolate4.restype = C.c_size_t
        L.ref_interpolate4.argtypes = [_u8p, _u8p]
        L.ref_poly_divide.argtypes = [_u8p, C.c_size_t, _u8p, C.c_size_t, _u8p,
                                      C.POINTER(C.c_size_t), _u8p, C.POINTER(C.c_size_t)]
        L.ref_plonk4_data.restype = C.c_size_t
        L.ref_plonk4_data.argtypes = [C.c_uint8, C.c_size_t, C.c_int] + [_u8p] * 6

    def plonk4_data(self, secret=2, srs_n=6, srs_mode=0):
        """srs_create + plonk_new(srs, 4): h, k1_h, k2_h, h_pows_inv (row-major), z_h_x, g1s."""
        h, k1, k2 = (np.zeros(4, np.uint8) for _ in range(3))
        hinv = np.zeros(16, np.uint8)
        zh = np.zeros(16, np.uint8)
        g1s = np.zeros(3 * (srs_n + 1), np.uint8)
        zl = self.lib.ref_plonk4_data(secret, srs_n, srs_mode, _ptr(h), _ptr(k1), _ptr(k2),
                                      _ptr(hinv), _ptr(zh), _ptr(g1s))
        return {"h": bytes(h), "k1_h": bytes(k1), "k2_h": bytes(k2), "h_pows_inv": bytes(hinv),
                "z_h": bytes(zh[:zl]), "g1s": bytes(g1s)}

    @staticmethod
    def available(path=os.path.join(HERE, "_ref", "libplonkref.so")):
        return os.path.exists(path)

    def msm(self, pts, sc):
        pts, sc = _u8(pts).reshape(-1), _u8(sc)
        assert pts.size == 3 * sc.size
        out = np.zeros(3, np.uint8)
        self.lib.ref_msm(_ptr(pts), _ptr(sc), sc.size, _ptr(out))
        return bytes(out)

    def poly_mul_ntt_blocked(self, a, b, piece):
        """orc_poly_mul_ntt_blocked: the shorter operand in pieces of at most `piece` coefficients"""
        a, b = _u8(a), _u8(b)
        out = np.zeros(len(a) + len(b) - 1, np.uint8)
        n = self.lib.orc_poly_mul_ntt_blocked(_ptr(a), len(a), _ptr(b), len(b), _ptr(out), int(piece))
        if n == 0:
            raise ValueError("orc_poly_mul_ntt_blocked: bad arguments")
        return bytes(out[:n])

    def poly_divide(self, num, den):
        num, den = _u8(num), _u8(den)
        q = np.zeros(max(len(num), 1), np.uint8)
        r = np.zeros(max(len(num), 1), np.uint8)
        lq, lr = C.c_size_t(), C.c_size_t()
        self.lib.ref_poly_divide(_ptr(num), len(num), _ptr(den), len(den), _ptr(q),
                                 C.byref(lq), _ptr(r), C.byref(lr))
        return bytes(q[:lq.value]), bytes(r[:lr.value])

    def interpolate4(self, values):
        out = np.zeros(4, np.uint8)
        n = self.lib.ref_interpolate4(_ptr(_u8(values)), _ptr(out))
        return bytes(out[:n])

    def prove4_inproc(self, gates, copies, wires, chal, rnd, secret=2, srs_n=6, srs_mode=0):
        """in-process prove (no fork): valid instances only (timing)"""
        f = self.lib.ref_prove4_inproc
        f.restype = None
        f.argtypes = [_u8p, _u8p, _u8p, _u8p, _u8p, C.c_uint8, C.c_size_t, C.c_int, _u8p]
        out = np.zeros(34, np.uint8)
        f(_ptr(_u8(gates)), _ptr(_u8(copies)), _ptr(_u8(wires)), _ptr(_u8(chal)), _ptr(_u8(rnd)), secret, srs_n,
          srs_mode, _ptr(out))
        return bytes(out)

    def prove4(self, gates, copies, wires, chal, rnd, secret=2, srs_n=6, srs_mode=0):
        out = np.zeros(34, np.uint8)
        rc = self.lib.ref_prove4(_ptr(_u8(gates)), _ptr(_u8(copies)), _ptr(_u8(wires)),
                                 _ptr(_u8(chal)), _ptr(_u8(rnd)), secret, srs_n, srs_mode,
                                 _ptr(out))
        return None if rc != 0 else bytes(out)
