#!/usr/bin/env python3
"""Golden answer of rounds 1-5 at n = 2^20 gates (config C5) from the CPU oracle
(oracle/prove_ref.py over oracle.c): the prove-shaped synthetic instance of
tests/test_prove_gpu.py::_synthetic with a fixed seed, non-strict (synthetic polynomials leave
remainders).  Writes tests/golden/prove_2_20.json (seed, n, srs_len, proof hex).
    python tests/golden/make_prove_2_20.py [log2n]"""
import json
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [HERE, os.path.join(ROOT, "oracle")]
import numpy as np  # noqa: E402

import gen  # noqa: E402
from prove_ref import Prover as RefProver  # noqa: E402
from pyoracle import Oracle  # noqa: E402

SEED = 51


def main():
    k = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    n = 1 << k
    srs_len = 2 * n + 8
    polys, chal, rnd, zh, pts = gen.prove_instance(n, SEED, srs_len)
    t = time.time()
    ref = RefProver(Oracle(), pts.tobytes(), n, z_h=zh.tobytes())
    proof = ref.rounds(polys, chal, rnd, strict=False)
    dt = time.time() - t
    out = {"seed": SEED, "n": n, "srs_len": srs_len, "proof": proof.hex(), "oracle_seconds": round(dt, 1),
           "note": "rounds 1-5 (plonk_prove, src/plonk.h:223-656) of the synthetic instance, CPU oracle"}
    name = "prove_2_20.json" if k == 20 else "prove_2_%d.json" % k
    with open(os.path.join(HERE, name), "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
