"""The drop-in headers' small-size policy (include/plk_host.h), on the CPU.

Calls whose host cost estimate is at most PLK_OPT_DROPIN_HOST_WORK stay on the host; larger
calls go to libplonkhip.  The host code is product code of the drop-in (not the oracle), so it is
pinned here the same way the GPU path is:
* the reference's own goldens (tests/golden: MSM cases incl. irregular encodings, poly_mul,
  poly_divide / poly_eval / matrix cases, the 26 toy proofs and interpolate_at_h) through the
  drop-in build of ref_harness.c (oracle/_ref/libplonkref_dropin.so) with the threshold raised so
  that every call runs on the host;
* live against the reference compiled from its unmodified headers (oracle/_ref/libplonkref.so)
  on seeded raw-byte inputs (every byte value, not only canonical residues);
* at the DEFAULT threshold the reference's own poly / srs / matrix / plonk test programs pass with
  no GPU visible (tests/test_reference_suite.py), and a call above the threshold still fails loudly
  without a GPU (no CPU fallback: the side a call runs on depends on its size only).
No GPU is touched: libplonkhip is loaded (the threshold is its option) but never initialised."""
import os
import subprocess
import sys

import numpy as np
import pytest

import gen
from conftest import ROOT, load_golden

DROPIN = os.path.join(ROOT, "oracle", "_ref", "libplonkref_dropin.so")
REFLIB = os.path.join(ROOT, "oracle", "_ref", "libplonkref.so")
EVERYTHING = 1 << 40


@pytest.fixture(scope="module")
def libs():
    for p in (DROPIN, REFLIB):
        assert os.path.exists(p), "%s missing: `make -C oracle` where /root/reference exists" % p
    import plonkhip
    from pyoracle import Reference
    D, R = Reference(DROPIN), Reference(REFLIB)
    with plonkhip.options(DROPIN_HOST_WORK=EVERYTHING):
        yield D, R


def test_default_threshold():
    import plonkhip
    assert plonkhip.get_option("DROPIN_HOST_WORK") == 32768


def test_goldens_on_the_host_path(libs):
    D, _ = libs
    m = load_golden("msm.json")
    for c in m["cases"] + m["irregular"]:
        pts = np.frombuffer(bytes.fromhex(c["points"]), np.uint8)
        sc = np.frombuffer(bytes.fromhex(c["scalars"]), np.uint8)
        assert D.msm(pts, sc).hex() == c["out"], c.get("kind")
    for c in load_golden("poly_mul.json")["cases"]:
        assert D.poly_mul(bytes.fromhex(c["a"]), bytes.fromhex(c["b"])).hex() == c["out"], c.get("note")
    g = load_golden("polyops.json")
    for c in g["divide"] + load_golden("poly_next.json")["divide"]:
        q, r = D.poly_divide(bytes.fromhex(c["num"]), bytes.fromhex(c["den"]))
        assert (q.hex(), r.hex()) == (c["q"], c["r"]), c.get("note", c["den"])
    for c in g["eval"] + load_golden("poly_next.json")["eval"]:
        assert D.poly_eval(bytes.fromhex(c["p"]), int(c["x"])) == int(c["y"]), c.get("note")
    for c in g["matrix_inv"]:
        assert D.matrix_inv(bytes.fromhex(c["m"]), int(c["n"])).hex() == c["inv"], c["note"]
    for c in g["matrix_mul"]:
        a, b = bytes.fromhex(c["a"]), bytes.fromhex(c["b"])
        assert D.matrix_mul(a, int(c["m"]), int(c["k"]), b, int(c["n"])).hex() == c["out"]
    p = load_golden("prove.json")
    for c in p["interpolate_at_h"]:
        assert D.interpolate4(c["values"]).hex() == c["out"]
    for c in p["proofs"]:
        args = (c["gates"], c["copies"], c["wires"], c["chal"], c["rand"], c["secret"], c["srs_n"], c["srs_mode"])
        assert D.prove4_inproc(*args).hex() == c["proof"], c.get("note", c["chal"])


def test_raw_bytes_vs_compiled_reference(libs):
    """seeded inputs over every byte value (poly operands, evaluation points, MSM points and
    scalars) and ragged lengths: the host path equals the reference compiled in place"""
    D, R = libs
    rng = np.random.default_rng(0x5A11)
    for t in range(400):
        raw = t % 2 == 1
        la, lb = int(rng.integers(1, 60)), int(rng.integers(1, 60))
        a = rng.integers(0, 256 if raw else 17, la).astype(np.uint8)
        b = rng.integers(0, 256 if t % 4 == 3 else 17, lb).astype(np.uint8)
        if t % 7 == 0:
            a[-3:] = 0                                    # trailing zeros: the trimmed length
        assert D.poly_mul(a, b) == R.poly_mul(a, b), (t, la, lb)
        x = int(rng.integers(0, 256 if raw else 17))
        assert D.poly_eval(a, x) == R.poly_eval(a, x), t
        den = rng.integers(0, 17, int(rng.integers(1, 8))).astype(np.uint8)
        den[-1] = int(rng.integers(1, 17))
        assert D.poly_divide(a, den) == R.poly_divide(a, den), (t, a.tolist(), den.tolist())
        n = int(rng.integers(0, 90))
        if raw:
            pts = rng.integers(0, 256, 3 * n).astype(np.uint8)
            pts[2::3] &= 1 if t % 3 else 0xFF             # flag bytes 0/1, sometimes any byte
            sc = rng.integers(0, 256, n).astype(np.uint8)
        else:                                             # all 102 group elements, scalars in [0, 16]
            pts, sc = gen.msm_inputs(t, n, "full")
        assert D.msm(pts, sc) == R.msm(pts, sc), (t, n)
        m, k, q = (int(v) for v in rng.integers(1, 7, 3))
        A = rng.integers(0, 256, m * k).astype(np.uint8)
        B = rng.integers(0, 256, k * q).astype(np.uint8)
        assert D.matrix_mul(A, m, k, B, q) == R.matrix_mul(A, m, k, B, q)
        M = rng.integers(0, 17, m * m).astype(np.uint8)
        assert D.matrix_inv(M, m) == R.matrix_inv(M, m)


def _run_child(code):
    """a child process with no GPU visible; returns (exit code, stderr)"""
    env = dict(os.environ, HIP_VISIBLE_DEVICES="-1", ROCR_VISIBLE_DEVICES="-1",
               PYTHONPATH=os.pathsep.join([os.path.join(ROOT, d) for d in ("plonk.c_amd", "oracle", "tests/golden")]))
    r = subprocess.run([sys.executable, "-c", code], cwd=ROOT, env=env, capture_output=True, text=True, timeout=120)
    return r.returncode, r.stderr


PRELUDE = ("import numpy as np, plonkhip\nfrom pyoracle import Reference\n"
           "D = Reference(%r)\n" % DROPIN)


def test_default_policy_boundary_without_a_gpu():
    """at the default threshold: a 181 x 181 product (32,761 <= 32,768) runs on the host with no
    GPU visible; 182 x 182 goes to libplonkhip and fails loudly (PLK_ERR_NODEV, the reference's
    stderr + exit convention); likewise a 109-point MSM (32,700) and a 110-point one"""
    rc, err = _run_child(PRELUDE + "a = np.ones(181, np.uint8)\nassert D.poly_mul(a, a)[:3] == bytes([1, 2, 3])\n"
                         "p = np.tile(np.array([1, 2, 0], np.uint8), 109)\n"
                         "assert D.msm(p, np.ones(109, np.uint8)) == D.msm(p[:3 * 7], np.ones(7, np.uint8))\n")
    assert rc == 0, err[-2000:]
    rc, err = _run_child(PRELUDE + "a = np.ones(182, np.uint8)\nD.poly_mul(a, a)\n")
    assert rc != 0 and "poly_mul failed on the GPU" in err and "no CPU fallback" in err, err[-2000:]
    rc, err = _run_child(PRELUDE + "p = np.tile(np.array([1, 2, 0], np.uint8), 110)\n"
                         "D.msm(p, np.ones(110, np.uint8))\n")
    assert rc != 0 and "srs_eval_at_s failed on the GPU" in err, err[-2000:]


def test_forced_gpu_policy_without_a_gpu():
    """threshold 0 (every call on the GPU): even a 2 x 2 product fails loudly without a device"""
    rc, err = _run_child(PRELUDE + "plonkhip.set_option('DROPIN_HOST_WORK', 0)\nD.poly_mul([1, 2], [3, 4])\n")
    assert rc != 0 and "poly_mul failed on the GPU" in err, err[-2000:]


def test_host_divide_rejects_raw_lead_like_the_library():
    rc, err = _run_child(PRELUDE + "D.poly_divide([1, 2, 3], [1, 20])\n")
    assert rc != 0 and "divisor lead byte 20 is not a GF(17) value" in err, err[-2000:]
