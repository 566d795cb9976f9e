"""Python plumbing over libplonkhip.so -- the C ABI declared in include/plonkhip.h.

The product boundary is the C ABI (and the drop-in C headers in include/ that the
reference's plonk.h compiles against).  This module only loads that library with ctypes
for the tests, bench.py and the multi-GPU driver; it never computes anything itself and
there is no fallback: if libplonkhip.so is missing or no GPU is usable, every call raises.

Host-buffer functions mirror the reference hot path (src/srs.h:53-68, src/poly.h:106-122):
    msm_g1(points, scalars) -> 3 bytes {x, y, infinite}        (srs_eval_at_s)
    poly_mul(a, b)          -> trimmed coefficient bytes         (poly_mul)
    srs_eval_at_s(g1s, coeffs) -- with the reference's degree check
Device functions take torch CUDA tensors (or raw ints) and an optional stream.
"""
import ctypes as C
import os

import numpy as np

PKG_DIR = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REPO_DIR = os.path.dirname(PKG_DIR)
LIB_PATH = os.environ.get("PLK_LIB") or os.path.join(PKG_DIR, "libplonkhip.so")   # PLK_LIB: tuning builds only
HEADER_PATH = os.path.join(REPO_DIR, "include", "plonkhip.h")

PLK_OK, PLK_ERR_HIP, PLK_ERR_ARG, PLK_ERR_RANGE, PLK_ERR_NODEV, PLK_ERR_NOMEM = range(6)
MSM_RESULT_BYTES = 2176
MSM_LOG_OFFSET, MSM_IRREGULAR_OFFSET, MSM_G1_OFFSET = 8, 12, 16

_u8p = C.POINTER(C.c_uint8)
_vp = C.c_void_p
_sz = C.c_size_t

# every exported entry point with its ctypes signature (restype, argtypes)
SIGNATURES = {
    "plk_init": (C.c_int, [C.c_int]),
    "plk_shutdown": (None, []),
    "plk_last_error": (C.c_char_p, []),
    "plk_device_count": (C.c_int, []),
    "plk_version": (C.c_char_p, []),
    "plk_msm_g1": (C.c_int, [_u8p, _u8p, _sz, _u8p]),
    "plk_poly_mul": (C.c_int, [_u8p, _sz, _u8p, _sz, _u8p, C.POINTER(_sz)]),
    "plk_msm_result_init": (C.c_int, [_vp, _vp]),
    "plk_msm_g1_dev": (C.c_int, [_vp, _vp, _sz, _vp, _vp]),
    "plk_msm_g1_batch_dev": (C.c_int, [_vp, _sz, _vp, _sz, _sz, C.c_int, _vp, _vp]),
    "plk_msm_g1_serial_dev": (C.c_int, [_vp, _vp, _sz, _vp, _vp]),
    "plk_msm_combine_dev": (C.c_int, [_vp, C.c_int, _vp, _vp]),
    "plk_msm_finalize_dev": (C.c_int, [_vp, C.c_int, C.c_int, _vp, _vp]),
    "plk_dlog_generator": (C.c_int, [_u8p]),
    "plk_poly_mul_workspace": (_sz, [_sz, _sz]),
    "plk_poly_mul_dev": (C.c_int, [_vp, _sz, _vp, _sz, _vp, _vp, _vp, _vp]),
    "plk_poly_mul_batch_workspace": (_sz, [_vp, C.c_int]),
    "plk_poly_mul_batch_dev": (C.c_int, [_vp, C.c_int, _vp, _sz, _vp]),
    "plk_ntt_dev": (C.c_int, [_vp, C.c_int, C.c_int, _vp]),
    "plk_ntt_batch_dev": (C.c_int, [_vp, C.c_int, C.c_int, C.c_int, _vp]),
    "plk_ntt29_dev": (C.c_int, [_vp, C.c_int, C.c_int, _vp]),
    "plk_ntt29_batch_dev": (C.c_int, [_vp, C.c_int, C.c_int, C.c_int, _vp]),
    "plk_poly_eval": (C.c_int, [_u8p, _sz, C.c_uint8, _u8p]),
    "plk_poly_eval_batch": (C.c_int, [C.POINTER(_u8p), C.POINTER(_sz), _u8p, C.c_int, _u8p]),
    "plk_poly_eval_workspace": (_sz, [C.c_int]),
    "plk_poly_eval_batch_dev": (C.c_int, [C.POINTER(_vp), C.POINTER(_sz), _u8p, C.c_int, _vp, _vp, _vp]),
    "plk_poly_divide": (C.c_int, [_u8p, _sz, _u8p, _sz, _u8p, C.POINTER(_sz), _u8p, C.POINTER(_sz)]),
    "plk_poly_divide_workspace": (_sz, [_sz, _sz]),
    "plk_poly_divide_dev": (C.c_int, [_vp, _sz, _u8p, _sz, _vp, _vp, _vp, _vp, _vp]),
    "plk_matrix_mul": (C.c_int, [_u8p, _sz, _sz, _u8p, _sz, _u8p]),
    "plk_matrix_inv": (C.c_int, [_u8p, _sz, _u8p]),
    "plk_interpolate": (C.c_int, [_u8p, _u8p, _sz, _u8p, C.POINTER(_sz)]),
    "plk_prover_create": (C.c_int, [_vp, C.POINTER(_vp)]),
    "plk_prover_destroy": (None, [_vp]),
    "plk_prover_device_bytes": (_sz, [_vp]),
    "plk_prover_prove": (C.c_int, [_vp, _vp, _u8p, _u8p, _u8p]),
    "plk_prover_rounds_dev": (C.c_int, [_vp, C.POINTER(_vp), _u8p, _u8p, C.c_int, _u8p]),
    "plk_prover_profile_dev": (C.c_int, [_vp, C.POINTER(_vp), _u8p, _u8p, C.c_int, _u8p, C.POINTER(C.c_double)]),
    "plk_prover_launches": (C.c_int, [_vp, C.POINTER(_vp), _u8p, _u8p, C.c_int, C.POINTER(C.c_int),
                                      C.POINTER(C.c_int)]),
    "plk_prover_alg_bytes": (C.c_uint64, [_vp]),
    "plk_prover_preprocess": (C.c_int, [_vp, C.POINTER(_vp)]),
    "plk_prover_chain_bytes": (_sz, [_vp, C.c_int]),
    "plk_prover_chains_dev": (C.c_int, [_vp, C.POINTER(_vp), _u8p, _u8p, C.c_int, _vp, _vp, _vp]),
    "plk_prover_rounds_ext_dev": (C.c_int, [_vp, C.POINTER(_vp), _u8p, _u8p, C.c_int, C.c_int, _vp, _vp, _vp,
                                            _u8p]),
    "plk_set_option": (C.c_int, [C.c_int, C.c_int64]),
    "plk_init_devices": (C.c_int, [C.POINTER(C.c_int), C.c_int]),
    "plk_devices": (C.c_int, [C.POINTER(C.c_int), C.c_int]),
    "plk_get_option": (C.c_int64, [C.c_int]),
    "plk_prover_attach_helpers": (C.c_int, [_vp, C.c_int]),
    "plk_prover_helpers": (C.c_int, [_vp]),
    "plk_prover_rounds_multi_dev": (C.c_int, [_vp, C.POINTER(_vp), C.c_int, _u8p, _u8p, C.c_int, _u8p]),
    "plk_ntt_launch_log": (C.c_int, [C.POINTER(C.c_int32), C.c_int]),
}

# PLK_OPT_* (include/plonkhip.h), by the name without the prefix
OPTIONS = {"TINY_CALLS": 1, "PROVE_SYNC": 2, "POLY_BLOCK_L": 3, "POLY_BLOCK_S": 4, "NTT_F29": 5, "NTT_SHARE": 6,
           "NTT_SHARED_FIX": 7, "NTT_T13_MIN_K": 8, "NTT_CENTER_BLOCKS": 9, "MSM_THREADS": 10,
           "MSM_MAX_BLOCKS": 11, "MSM_GROUPS": 12, "MSM_COPIES": 13, "MSM_HALF": 14, "MSM_SHARD_MIN": 15,
           "NTT_CENTER_SUM": 16, "MSM_HOST_LANES": 17,
           "PROVE_DERIVE_T2A": 18, "NTT_TABLE_SHARE": 19, "NTT_LAUNCH_LOG": 20,
           "PROVE_FUSE_DIV": 21, "PROVE_SRS_LOGS": 22,
           "PROVE_PACK_FUSE": 23, "PROVE_EARLY_COMMITS": 24,
           "PROVE_HELPER_COPY": 25, "PROVE_EVAL_AGG": 26, "PROVE_GRAPH": 27,
           "DROPIN_HOST_WORK": 28}

PLK_PROVE_STRICT = 1
PLK_PROVE_PREPROCESSED = 2
PLK_CHAIN_T2 = 1   # t_2 = (A2 B2)(C2 z_x), src/plonk.h:432-434
PLK_CHAIN_T3 = 2   # t_3 = (A3 B3)(C3 z_x(omega x)), src/plonk.h:471-473


class PlonkDesc(C.Structure):
    """plk_plonk_desc_t"""
    _fields_ = [("n", _sz), ("h", _u8p), ("k1_h", _u8p), ("k2_h", _u8p), ("h_pows_inv", _u8p),
                ("z_h", _u8p), ("z_h_len", _sz), ("srs_g1", _u8p), ("srs_len", _sz)]


class Circuit(C.Structure):
    """plk_circuit_t"""
    _fields_ = [(k, _u8p) for k in ("q_m", "q_l", "q_r", "q_o", "q_c", "copy_a", "copy_b",
                                    "copy_c", "a", "b", "c")]


class PlonkHipError(RuntimeError):
    def __init__(self, fn, code, msg):
        super().__init__("%s failed (code %d): %s" % (fn, code, msg))
        self.code = code


_lib = None


def lib():
    """Load libplonkhip.so (raises if it was never built)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise FileNotFoundError("libplonkhip.so not built (run `make -C plonk.c_amd` or "
                                    "__graft_entry__.build()): %s" % LIB_PATH)
        # torch-ROCm ships its own libamdhip64 (soname libamdhip64.so.7) and asks for it by a
        # different file name, so loading ours first would put TWO HIP runtimes in the
        # process.  Load torch first: our NEEDED libamdhip64.so.7 then binds to torch's copy
        # and the process has one runtime, one device context, shared streams.
        try:
            import torch  # noqa: F401
        except ImportError:
            pass
        L = C.CDLL(LIB_PATH)
        for name, (res, args) in SIGNATURES.items():
            f = getattr(L, name)
            f.restype = res
            f.argtypes = args
        _lib = L
    return _lib


def last_error():
    return lib().plk_last_error().decode(errors="replace")


def _check(fn, rc):
    if rc != PLK_OK:
        raise PlonkHipError(fn, rc, last_error())


def _u8(a):
    return np.ascontiguousarray(np.frombuffer(a, np.uint8) if isinstance(a, (bytes, bytearray))
                                else np.asarray(a, dtype=np.uint8))


def _p(a):
    return a.ctypes.data_as(_u8p)


def init(device=-1):
    _check("plk_init", lib().plk_init(int(device)))


def init_devices(ids):
    """plk_init_devices: ids[0] is the primary device; plk_msm_g1 point-range shards over the
    list (repeats allowed: several shards on one GPU)"""
    ids = [int(i) for i in ids]
    arr = (C.c_int * max(1, len(ids)))(*ids)
    _check("plk_init_devices", lib().plk_init_devices(arr, len(ids)))


def devices():
    arr = (C.c_int * 16)()
    n = int(lib().plk_devices(arr, 16))
    return [arr[i] for i in range(min(n, 16))]


def ntt_launch_log(cap=4096):
    """plk_ntt_launch_log: the recorded NTT pass launches (PLK_OPT_NTT_LAUNCH_LOG = 1) as dicts, log cleared"""
    buf = (C.c_int32 * (8 * cap))()
    n = int(lib().plk_ntt_launch_log(buf, cap))
    keys = ("kind", "tb", "m", "k", "n", "per_block", "units", "field")
    return [dict(zip(keys, buf[8 * i:8 * i + 8])) for i in range(n)]


def _opt_id(name):
    return OPTIONS[name.upper()] if isinstance(name, str) else int(name)


def set_option(name, value):
    """plk_set_option: name = "NTT_F29", ... (PLK_OPT_ without the prefix) or the number"""
    _check("plk_set_option", lib().plk_set_option(_opt_id(name), int(value)))


def get_option(name):
    return int(lib().plk_get_option(_opt_id(name)))


class options:
    """with options(NTT_F29=0, ...): set for the block, the previous values restored after"""

    def __init__(self, **kw):
        self.kw = kw
        self.old = {}

    def __enter__(self):
        for k, v in self.kw.items():
            self.old[k] = get_option(k)
            set_option(k, v)
        return self

    def __exit__(self, *exc):
        for k, v in self.old.items():
            set_option(k, v)
        return False


def tune_from_env():
    """bench / tools only (never called by the library or the tests' product path): apply
    $PLK_TUNE = "NAME=value,NAME=value" through plk_set_option, for A/B runs of one build.
    Returns the dict applied."""
    spec = os.environ.get("PLK_TUNE", "")
    done = {}
    for item in filter(None, (t.strip() for t in spec.split(","))):
        k, v = item.split("=")
        set_option(k.strip(), int(v))
        done[k.strip().upper()] = int(v)
    return done


def device_count():
    return int(lib().plk_device_count())


def dlog_generator():
    out = np.zeros(3, np.uint8)
    _check("plk_dlog_generator", lib().plk_dlog_generator(_p(out)))
    return bytes(out)


# ---------------------------------------------------------------- host-buffer entry points
def msm_g1(points, scalars):
    """sum_i scalars[i] * points[i] as the reference's serial fold would return it."""
    pts = _u8(points).reshape(-1)
    sc = _u8(scalars).reshape(-1)
    if pts.size != 3 * sc.size:
        raise ValueError("points must be n x 3 bytes for n scalars")
    out = np.zeros(3, np.uint8)
    _check("plk_msm_g1", lib().plk_msm_g1(_p(pts), _p(sc), sc.size, _p(out)))
    return bytes(out)


def srs_eval_at_s(g1s, coeffs):
    """srs_eval_at_s(srs, vs) (src/srs.h:53-68): the reference exits when the polynomial is
    longer than the SRS; this mirror raises ValueError instead of exiting the interpreter."""
    pts = _u8(g1s).reshape(-1)
    sc = _u8(coeffs).reshape(-1)
    if sc.size > pts.size // 3:
        raise ValueError("Poynomial degree exceeds SRS size: POLY degree: %d, SRS supports up "
                         "to degree: %d" % (sc.size, sc.size))
    return msm_g1(pts[:3 * sc.size], sc)


def poly_mul(a, b):
    """GF(17) product, trimmed exactly like the reference's poly_new."""
    a = _u8(a).reshape(-1)
    b = _u8(b).reshape(-1)
    rl = max(a.size + b.size - 1, 1)
    out = np.zeros(rl, np.uint8)
    n = _sz(0)
    _check("plk_poly_mul", lib().plk_poly_mul(_p(a), a.size, _p(b), b.size, _p(out), C.byref(n)))
    return bytes(out[:n.value])


def poly_eval(p, x):
    """Horner at x exactly as src/poly.h:265-272 (raw HF bytes included)."""
    p = _u8(p).reshape(-1)
    y = np.zeros(1, np.uint8)
    _check("plk_poly_eval", lib().plk_poly_eval(_p(p), p.size, int(x) & 0xFF, _p(y)))
    return int(y[0])


def poly_eval_batch(polys, xs):
    arrs = [_u8(p).reshape(-1) for p in polys]
    n = len(arrs)
    ptrs = (_u8p * n)(*[_p(a) for a in arrs])
    lens = (_sz * n)(*[a.size for a in arrs])
    xa = _u8(xs).reshape(-1)
    ys = np.zeros(n, np.uint8)
    _check("plk_poly_eval_batch", lib().plk_poly_eval_batch(ptrs, lens, _p(xa), n, _p(ys)))
    return [int(v) for v in ys]


def poly_divide(num, den):
    """(quot, rem) bytes, trimmed as src/poly.h:124-177 returns them."""
    num = _u8(num).reshape(-1)
    den = _u8(den).reshape(-1)
    q = np.zeros(max(num.size, 1), np.uint8)
    r = np.zeros(max(num.size, 1), np.uint8)
    ql, rl = _sz(0), _sz(0)
    _check("plk_poly_divide", lib().plk_poly_divide(_p(num), num.size, _p(den), den.size, _p(q), C.byref(ql),
                                                    _p(r), C.byref(rl)))
    return bytes(q[:ql.value]), bytes(r[:rl.value])


def matrix_mul(a, m, k, b, n):
    a = _u8(a).reshape(-1)
    b = _u8(b).reshape(-1)
    out = np.zeros(max(m * n, 1), np.uint8)
    _check("plk_matrix_mul", lib().plk_matrix_mul(_p(a), m, k, _p(b), n, _p(out)))
    return bytes(out[:m * n])


def matrix_inv(mat, n):
    mat = _u8(mat).reshape(-1)
    out = np.zeros(max(n * n, 1), np.uint8)
    _check("plk_matrix_inv", lib().plk_matrix_inv(_p(mat), n, _p(out)))
    return bytes(out[:n * n])


def interpolate(h_pows_inv, values):
    v = _u8(values).reshape(-1)
    m = _u8(h_pows_inv).reshape(-1)
    out = np.zeros(max(v.size, 1), np.uint8)
    ol = _sz(0)
    _check("plk_interpolate", lib().plk_interpolate(_p(m), _p(v), v.size, _p(out), C.byref(ol)))
    return bytes(out[:ol.value])


# ---------------------------------------------------------------- device entry points
def _ptr(t):
    if t is None:
        return None
    if isinstance(t, int):
        return t
    return t.data_ptr()


def _stream(s):
    if s is None:
        return None
    if isinstance(s, int):
        return s
    return s.cuda_stream


def msm_result_init(res, stream=None):
    _check("plk_msm_result_init", lib().plk_msm_result_init(_ptr(res), _stream(stream)))


def msm_g1_dev(points, scalars, n, res, stream=None):
    _check("plk_msm_g1_dev", lib().plk_msm_g1_dev(_ptr(points), _ptr(scalars), int(n), _ptr(res),
                                                  _stream(stream)))


def msm_g1_batch_dev(points, points_stride, scalars, scalars_stride, n, batch, res, stream=None):
    _check("plk_msm_g1_batch_dev", lib().plk_msm_g1_batch_dev(
        _ptr(points), int(points_stride), _ptr(scalars), int(scalars_stride), int(n), int(batch),
        _ptr(res), _stream(stream)))


def msm_g1_serial_dev(points, scalars, n, res, stream=None):
    _check("plk_msm_g1_serial_dev", lib().plk_msm_g1_serial_dev(_ptr(points), _ptr(scalars), int(n),
                                                                _ptr(res), _stream(stream)))


def msm_combine_dev(logs, count, out3, stream=None):
    _check("plk_msm_combine_dev", lib().plk_msm_combine_dev(_ptr(logs), int(count), _ptr(out3),
                                                            _stream(stream)))


def msm_finalize_dev(logs, batch, stride, out4, stream=None):
    _check("plk_msm_finalize_dev", lib().plk_msm_finalize_dev(_ptr(logs), int(batch), int(stride),
                                                              _ptr(out4), _stream(stream)))


def poly_mul_workspace(la, lb):
    return int(lib().plk_poly_mul_workspace(int(la), int(lb)))


def poly_mul_dev(a, la, b, lb, out, nz, work, stream=None):
    _check("plk_poly_mul_dev", lib().plk_poly_mul_dev(_ptr(a), int(la), _ptr(b), int(lb), _ptr(out),
                                                      _ptr(nz), _ptr(work), _stream(stream)))


class PolyMulJob(C.Structure):
    """plk_polymul_job_t (include/plonkhip.h)"""
    _fields_ = [("a", C.c_void_p), ("la", C.c_size_t), ("b", C.c_void_p), ("lb", C.c_size_t),
                ("out", C.c_void_p), ("acc", C.c_int)]


def _jobs(jobs):
    arr = (PolyMulJob * len(jobs))()
    for i, (a, la, b, lb, out, acc) in enumerate(jobs):
        arr[i] = PolyMulJob(_ptr(a), int(la), _ptr(b), int(lb), _ptr(out), int(acc))
    return arr


def poly_mul_batch_workspace(jobs):
    """jobs: (a, la, b, lb, out, acc) tuples of device tensors / pointers"""
    arr = _jobs(jobs)
    return int(lib().plk_poly_mul_batch_workspace(arr, len(jobs)))


def poly_mul_batch_dev(jobs, work, work_bytes, stream=None):
    arr = _jobs(jobs)
    _check("plk_poly_mul_batch_dev", lib().plk_poly_mul_batch_dev(arr, len(jobs), _ptr(work), int(work_bytes),
                                                                  _stream(stream)))


def poly_eval_workspace(n):
    return int(lib().plk_poly_eval_workspace(int(n)))


def poly_eval_batch_dev(polys, lens, xs, ys, tick, stream=None):
    """polys: device tensors (or raw pointers); tick: zeroed device workspace."""
    n = len(polys)
    ptrs = (_vp * n)(*[_ptr(p) for p in polys])
    ls = (_sz * n)(*[int(v) for v in lens])
    xa = _u8(xs).reshape(-1)
    _check("plk_poly_eval_batch_dev", lib().plk_poly_eval_batch_dev(ptrs, ls, _p(xa), n, _ptr(ys), _ptr(tick),
                                                                    _stream(stream)))


def poly_divide_workspace(nl, dl):
    return int(lib().plk_poly_divide_workspace(int(nl), int(dl)))


def poly_divide_dev(num, nl, den, quot, rem, lens, work, stream=None):
    """den: HOST bytes (classified on the host)."""
    d = _u8(den).reshape(-1)
    _check("plk_poly_divide_dev", lib().plk_poly_divide_dev(_ptr(num), int(nl), _p(d), d.size, _ptr(quot),
                                                            _ptr(rem), _ptr(lens), _ptr(work), _stream(stream)))


def ntt_dev(data, log_n, inverse=False, stream=None):
    _check("plk_ntt_dev", lib().plk_ntt_dev(_ptr(data), int(log_n), 1 if inverse else 0,
                                            _stream(stream)))


def ntt_batch_dev(data, log_n, batch, inverse=False, stream=None):
    _check("plk_ntt_batch_dev", lib().plk_ntt_batch_dev(_ptr(data), int(log_n), int(batch), 1 if inverse else 0,
                                                        _stream(stream)))


def ntt29_dev(data, log_n, inverse=False, stream=None):
    """plk_ntt29_dev: the same transform over F29 (p = 7 2^26 + 1), log_n 13..26."""
    _check("plk_ntt29_dev", lib().plk_ntt29_dev(_ptr(data), int(log_n), 1 if inverse else 0, _stream(stream)))


def ntt29_batch_dev(data, log_n, batch, inverse=False, stream=None):
    _check("plk_ntt29_batch_dev", lib().plk_ntt29_batch_dev(_ptr(data), int(log_n), int(batch),
                                                            1 if inverse else 0, _stream(stream)))


def parse_result(res_bytes):
    """Decode a plk_msm_result_t (MSM_RESULT_BYTES) copied to the host."""
    b = bytes(res_bytes)
    return {"log": int.from_bytes(b[MSM_LOG_OFFSET:MSM_LOG_OFFSET + 4], "little"),
            "irregular": int.from_bytes(b[MSM_IRREGULAR_OFFSET:MSM_IRREGULAR_OFFSET + 4], "little"),
            "g1": b[MSM_G1_OFFSET:MSM_G1_OFFSET + 3]}


# ---------------------------------------------------------------- device prover
class Prover:
    """plk_prover_t: plonk_new's setup on the device (SRS + Z_H [+ circuit tables]),
    plonk_prove as `prove` (circuit) or `rounds_dev` (device-resident interpolated polys)."""

    def __init__(self, n, z_h, srs_g1, h=None, k1_h=None, k2_h=None, h_pows_inv=None):
        self._keep = [_u8(x) if x is not None else None for x in (h, k1_h, k2_h, h_pows_inv, z_h, srs_g1)]
        hh, k1, k2, hi, zh, srs = self._keep
        d = PlonkDesc(n, *(None if x is None else _p(x) for x in (hh, k1, k2, hi)), _p(zh), zh.size,
                      _p(srs), srs.size // 3)
        self._h = _vp()
        _check("plk_prover_create", lib().plk_prover_create(C.byref(d), C.byref(self._h)))
        self.n = n

    def close(self):
        if self._h:
            lib().plk_prover_destroy(self._h)
            self._h = _vp()
        self._fixed = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def device_bytes(self):
        return int(lib().plk_prover_device_bytes(self._h))

    def prove(self, q_m, q_l, q_r, q_o, q_c, copy_a, copy_b, copy_c, a, b, c, chal, rand):
        """copy_*: n (type, index) pairs, flattened or not."""
        arrs = [_u8(x).reshape(-1) for x in (q_m, q_l, q_r, q_o, q_c, copy_a, copy_b, copy_c, a, b, c)]
        cir = Circuit(*(_p(x) for x in arrs))
        ch, rd = _u8(chal), _u8(rand)
        out = np.zeros(34, np.uint8)
        _check("plk_prover_prove", lib().plk_prover_prove(self._h, C.byref(cir), _p(ch), _p(rd), _p(out)))
        return bytes(out)

    def _args(self, polys, chal, rand):
        """ctypes argument blocks of (polys, chal, rand), cached by value"""
        cache = self.__dict__.setdefault("_argcache", {})
        ch, rd = _u8(chal).reshape(-1), _u8(rand).reshape(-1)
        if ch.size != 5 or rd.size != 9:
            raise ValueError("rounds_dev: chal must hold 5 values and rand 9 (got %d, %d)" % (ch.size, rd.size))
        if len(polys) != 13:
            raise ValueError("rounds_dev: 13 polynomials, got %d" % len(polys))
        key = (tuple(p if isinstance(p, int) else p.data_ptr() for p in polys), ch.tobytes(), rd.tobytes())
        args = cache.get(key)
        if args is None:
            if len(cache) > 64:
                cache.clear()
            args = ((_vp * 13)(*key[0]), (C.c_uint8 * 5).from_buffer_copy(key[1]),
                    (C.c_uint8 * 9).from_buffer_copy(key[2]))
            cache[key] = args
        return args

    def rounds_dev(self, polys, chal, rand, strict=False, preprocessed=False):
        """polys: 13 device tensors / pointers (n bytes each).  preprocessed: use the fixed
        polynomials' transforms from `preprocess` (same addresses, unchanged bytes).  The ctypes
        argument blocks are cached by value (a 2^20-gate proof is ~0.5 ms: building them anew
        each call was ~5 % of it)."""
        args = self._args(polys, chal, rand)
        out = self.__dict__.setdefault("_out", (C.c_uint8 * 34)())
        flags = (PLK_PROVE_STRICT if strict else 0) | (PLK_PROVE_PREPROCESSED if preprocessed else 0)
        _check("plk_prover_rounds_dev", lib().plk_prover_rounds_dev(self._h, args[0], args[1], args[2], flags, out))
        return bytes(out)

    def profile_dev(self, polys, chal, rand, preprocessed=False):
        """plk_prover_profile_dev: (proof bytes, {span_ms, ntt_ms, batch1_ms, batch2_ms}) -- the proof's
        launch sequence and its two product batches (all its NTT pass kernels) timed by hipEvents on the
        prover's stream"""
        args = self._args(polys, chal, rand)
        out = (C.c_uint8 * 34)()
        ms = (C.c_double * 4)()
        flags = PLK_PROVE_PREPROCESSED if preprocessed else 0
        _check("plk_prover_profile_dev",
               lib().plk_prover_profile_dev(self._h, args[0], args[1], args[2], flags, out, ms))
        return bytes(out), dict(zip(("span_ms", "ntt_ms", "batch1_ms", "batch2_ms"), list(ms)))

    def launches(self, polys, chal, rand, preprocessed=False):
        """plk_prover_launches: (kernel launches, other graph nodes) of one proof, counted from a
        captured (never launched) HIP graph of the call"""
        args = self._args(polys, chal, rand)
        k, o = C.c_int(), C.c_int()
        flags = PLK_PROVE_PREPROCESSED if preprocessed else 0
        _check("plk_prover_launches",
               lib().plk_prover_launches(self._h, args[0], args[1], args[2], flags, C.byref(k), C.byref(o)))
        return k.value, o.value

    def alg_bytes(self):
        """plk_prover_alg_bytes: the proof's algorithmic bytes in SURVEY 8(d) terms"""
        return int(lib().plk_prover_alg_bytes(self._h))

    # ---- strong-scaled proof (plk_prover_chains_dev / plk_prover_rounds_ext_dev)
    def chain_bytes(self, chain):
        """buffer size for one chain's product (PLK_CHAIN_T2 or PLK_CHAIN_T3)"""
        return int(lib().plk_prover_chain_bytes(self._h, int(chain)))

    def _check_chain_bufs(self, which, t2, t3):
        """a chain buffer in `which` must be a device tensor of at least chain_bytes on this
        prover's device (an undersized one would be written / read past its end on the GPU);
        raw integer pointers are passed through unchecked"""
        for chain, t in ((PLK_CHAIN_T2, t2), (PLK_CHAIN_T3, t3)):
            if not (int(which) & chain) or t is None or isinstance(t, int):
                continue
            need = self.chain_bytes(chain)
            have = t.numel() * t.element_size()
            if have < need:
                raise ValueError("chain %d buffer holds %d bytes, chain_bytes is %d" % (chain, have, need))
            if not t.is_cuda:
                raise ValueError("chain %d buffer is not a device tensor" % chain)
            dev = getattr(self, "device", None)
            if dev is not None and t.device.index != dev:
                raise ValueError("chain %d buffer is on device %s, the prover on %d" % (chain, t.device, dev))

    def chains_dev(self, polys, chal, rand, which, t2=None, t3=None, done=None):
        """Helper GPU: enqueue the preparation and the chains in `which` (PLK_CHAIN_* mask) into
        the device buffers t2 / t3 (chain_bytes each); stream `done` (None: the null stream,
        torch's default) waits for them."""
        self._check_chain_bufs(which, t2, t3)
        args = self._args(polys, chal, rand)
        _check("plk_prover_chains_dev", lib().plk_prover_chains_dev(
            self._h, args[0], args[1], args[2], int(which), _ptr(t2) if t2 is not None else None,
            _ptr(t3) if t3 is not None else None, _stream(done)))

    def rounds_ext_dev(self, polys, chal, rand, which, t2=None, t3=None, ready=None, strict=False,
                       preprocessed=False):
        """rounds_dev with the chains in `which` read from t2 / t3 (computed by chains_dev on
        another GPU from the same inputs) once everything enqueued on stream `ready` (None: the
        null stream) so far has run.  Same 34 bytes as rounds_dev."""
        self._check_chain_bufs(which, t2, t3)
        args = self._args(polys, chal, rand)
        out = (C.c_uint8 * 34)()
        flags = (PLK_PROVE_STRICT if strict else 0) | (PLK_PROVE_PREPROCESSED if preprocessed else 0)
        _check("plk_prover_rounds_ext_dev", lib().plk_prover_rounds_ext_dev(
            self._h, args[0], args[1], args[2], flags, int(which), _ptr(t2) if t2 is not None else None,
            _ptr(t3) if t3 is not None else None, _stream(ready), out))
        return bytes(out)

    # ---- the same split from C over the plk_init_devices list (plk_prover_attach_helpers)
    def attach_helpers(self, k):
        """k helper provers on entries 1..k of the plk_init_devices list (0 detaches); from then on
        rounds_dev / prove run split (the chains on the helpers, products peer-copied back)"""
        _check("plk_prover_attach_helpers", lib().plk_prover_attach_helpers(self._h, int(k)))

    def helpers(self):
        return int(lib().plk_prover_helpers(self._h))

    def rounds_multi_dev(self, poly_sets, chal, rand, strict=False, preprocessed=False):
        """poly_sets: 1 + helpers() lists of 13 device tensors, set h on helper h's device"""
        ch, rd = _u8(chal).reshape(-1), _u8(rand).reshape(-1)
        if ch.size != 5 or rd.size != 9:
            raise ValueError("rounds_multi_dev: chal must hold 5 values and rand 9")
        flat = [p for ps in poly_sets for p in ps]
        if any(len(ps) != 13 for ps in poly_sets):
            raise ValueError("rounds_multi_dev: 13 polynomials per set")
        arr = (_vp * len(flat))(*[_ptr(p) for p in flat])
        out = (C.c_uint8 * 34)()
        flags = (PLK_PROVE_STRICT if strict else 0) | (PLK_PROVE_PREPROCESSED if preprocessed else 0)
        _check("plk_prover_rounds_multi_dev", lib().plk_prover_rounds_multi_dev(
            self._h, arr, len(poly_sets), _p(ch), _p(rd), flags, out))
        return bytes(out)

    def preprocess(self, polys):
        """plk_prover_preprocess: the round-3 transforms of q_o q_m q_l q_r s_sigma_3 l_1_x
        (entries 3 4 5 6 10 12 of the 13 device polys); None drops them."""
        arr = None if polys is None else (_vp * 13)(*[_ptr(p) for p in polys])
        # the transforms are bound to these device addresses: hold the tensors so the caching
        # allocator cannot hand the same addresses to another circuit's polynomials
        self._fixed = None
        _check("plk_prover_preprocess", lib().plk_prover_preprocess(self._h, arr))
        self._fixed = None if polys is None else list(polys)
