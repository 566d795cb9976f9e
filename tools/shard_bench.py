"""plk_msm_g1 (host buffers, what srs_eval_at_s calls) over 1..N shards of device 0 (or the
devices given): wall time per call with the SRS cached and re-uploaded, 2^20 and 2^22 points."""
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "plonk.c_amd"))
import plonkhip as hip  # noqa: E402

hip.tune_from_env()   # PLK_TUNE="NAME=value,..." (plk_set_option), tuning runs only
hip.init(0)
ndev = hip.device_count()
out = {}
rng = np.random.default_rng(3)
kg = np.array([[1, 2, 0], [68, 74, 0], [26, 45, 0], [65, 98, 0]], np.uint8)
for log2n in (20, 22):
    n = 1 << log2n
    pts = kg[rng.integers(0, 4, n)].reshape(-1)
    sc = rng.integers(0, 17, n, dtype=np.uint8)
    for ns in (1, 2, 4, 8):
        ids = [i % ndev for i in range(ns)]
        hip.init_devices(ids)
        want = hip.msm_g1(pts, sc)
        t0 = time.perf_counter()
        for _ in range(10):
            assert hip.msm_g1(pts, sc) == want
        cached = (time.perf_counter() - t0) / 10 * 1e6
        copies = [pts.copy() for _ in range(5)]
        t0 = time.perf_counter()
        for c in copies:
            assert hip.msm_g1(c, sc) == want
        fresh = (time.perf_counter() - t0) / 5 * 1e6
        out["2^%d_shards%d" % (log2n, ns)] = {"devices": ids, "srs_cached_us": round(cached, 1),
                                              "srs_uploaded_us": round(fresh, 1)}
hip.init_devices([0])
print(json.dumps(out))
