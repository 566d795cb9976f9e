"""Drop-in proof: the reference's UNMODIFIED plonk.h prover compiled against include/
(pre-included prelude) so poly_mul / srs_eval_at_s run in libplonkhip on the GPU.  The
34-byte proofs must equal the golden proofs recorded from the all-CPU reference -- with the
small-size policy at its default (toy calls on the host, include/plk_host.h) and at 0 (every
call on the GPU, PLK_OPT_DROPIN_HOST_WORK).

The drop-in library (oracle/_ref/libplonkref_dropin.so) can only be BUILT where
/root/reference exists; it travels to the GPU box with the snapshot (oracle/_ref is git-ignored,
not gpurun-ignored).  A missing build FAILS these tests, as in test_reference_suite.py: a silent
skip would hide that the drop-in was never exercised."""
import os

import numpy as np
import pytest

import gen
from conftest import ROOT, load_golden

pytestmark = pytest.mark.gpu
DROPIN = os.path.join(ROOT, "oracle", "_ref", "libplonkref_dropin.so")


@pytest.fixture(scope="module", params=["default", "all_gpu"])
def dropin(hip, request):
    assert os.path.exists(DROPIN), ("drop-in build absent: %s (make -C oracle, needs /root/reference at "
                                    "build time; it travels to the GPU box in the snapshot)" % DROPIN)
    from pyoracle import Reference
    if request.param == "default":
        yield Reference(DROPIN)
    else:
        with hip.options(DROPIN_HOST_WORK=0):
            yield Reference(DROPIN)


def test_toy_proof_bytes(dropin):
    g = load_golden("prove.json")
    for p in g["proofs"]:
        got = dropin.prove4(p["gates"], p["copies"], p["wires"], p["chal"], p["rand"],
                            p["secret"], p["srs_n"], p["srs_mode"])
        assert got.hex() == p["proof"], p.get("note", p["chal"])


def test_interpolate_and_hot_ops(dropin):
    g = load_golden("prove.json")
    for c in g["interpolate_at_h"]:
        assert dropin.interpolate4(c["values"]).hex() == c["out"]
    for c in load_golden("msm.json")["cases"]:
        pts = np.frombuffer(bytes.fromhex(c["points"]), np.uint8)
        sc = np.frombuffer(bytes.fromhex(c["scalars"]), np.uint8)
        assert dropin.msm(pts, sc).hex() == c["out"]
    for c in load_golden("poly_mul.json")["cases"]:
        assert dropin.poly_mul(bytes.fromhex(c["a"]), bytes.fromhex(c["b"])).hex() == c["out"]


def test_large_through_headers(dropin):
    c = load_golden("msm.json")["large"][5]
    pts, sc = gen.msm_inputs(c["seed"], c["n"], c["kind"])
    assert dropin.msm(pts, sc).hex() == c["out"]
    c = load_golden("poly_mul.json")["large"][6]
    a, b = gen.poly_inputs(c["seed"], c["la"], c["lb"])
    out = dropin.poly_mul(a, b)
    assert gen.digest(np.frombuffer(out, np.uint8)) == c["sha256"]


def test_both_sides_of_the_small_size_threshold(hip):
    """The drop-in's small-size policy (include/plk_host.h) at its default: calls just below the
    threshold run on the host, calls just above it on the GPU -- both equal to the reference compiled
    in place (oracle/_ref/libplonkref.so), on canonical and raw bytes"""
    from pyoracle import Reference
    D, R = Reference(DROPIN), Reference()
    # (the default, set explicitly: the module's parametrized fixture may still hold the all-GPU
    # setting; tests/test_dropin_host_cpu.py checks the library's default itself)
    with hip.options(DROPIN_HOST_WORK=32768):
        _threshold_cases(D, R)


def _threshold_cases(D, R):
    rng = np.random.default_rng(21)
    for la, lb in ((181, 181), (182, 182), (32768, 1), (32769, 1), (100, 400), (100, 500)):
        for mod in (17, 256):
            a = rng.integers(0, mod, la).astype(np.uint8)
            b = rng.integers(0, mod, lb).astype(np.uint8)
            assert D.poly_mul(a, b) == R.poly_mul(a, b), (la, lb, mod)
    for n in (109, 110, 3000):                        # 300 n: host up to 109 points
        pts, sc = gen.msm_inputs(n, n, "full")
        assert D.msm(pts, sc) == R.msm(pts, sc), n
    for nl, dl in ((4000, 4), (4200, 4), (9000, 2)):   # 2 (nl - dl + 1) dl around 32768
        num = rng.integers(0, 17, nl).astype(np.uint8)
        den = rng.integers(0, 17, dl).astype(np.uint8)
        den[-1] = 5
        assert D.poly_divide(num, den) == R.poly_divide(num, den), (nl, dl)
    for ln in (16384, 16385, 100000):                 # 2 len around 32768
        p = rng.integers(0, 256, ln).astype(np.uint8)
        assert D.poly_eval(p, 7) == R.poly_eval(p, 7), ln
