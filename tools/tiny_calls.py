#!/usr/bin/env python3
"""Per-call latency of the host-buffer C ABI at toy sizes (what the drop-in headers call from the
reference's 4-gate prove): microseconds per call, 500 calls each (tuning aid)."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "plonk.c_amd"))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402,F401  (one HIP runtime per process)

import plonkhip as hip  # noqa: E402

hip.tune_from_env()   # PLK_TUNE="NAME=value,..." (plk_set_option), tuning runs only
hip.init(0)
rng = np.random.default_rng(1)
p8 = rng.integers(0, 17, 8, dtype=np.uint8)
q8 = rng.integers(0, 17, 8, dtype=np.uint8)
pts = np.tile(np.array([1, 2, 0], np.uint8), 8)
sc = rng.integers(0, 17, 8, dtype=np.uint8)
m4 = rng.integers(0, 17, 16, dtype=np.uint8)
den = np.array([16, 1], np.uint8)
calls = {
    "poly_eval_8": lambda: hip.poly_eval(p8, 3),
    "poly_mul_8x8": lambda: hip.poly_mul(p8, q8),
    "msm_g1_8": lambda: hip.msm_g1(pts, sc),
    "poly_divide_8_by_2": lambda: hip.poly_divide(p8, den),
    "matrix_mul_4x4": lambda: hip.matrix_mul(m4, 4, 4, m4, 4),
}
out = {}
for name, fn in calls.items():
    for _ in range(20):
        fn()
    t0 = time.perf_counter()
    for _ in range(500):
        fn()
    out[name + "_us"] = round((time.perf_counter() - t0) / 500 * 1e6, 2)
print(json.dumps(out))
