"""plk_msm_g1 over every visible GPU (plk_init_devices with distinct device ids): the multi-device
host-buffer path of srs_eval_at_s at 2^22 points, against device 0 alone.  Run by bench.py as a
child process (its own contexts, a time limit) on multi-GPU nodes; prints one JSON object."""
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "plonk.c_amd"))
import plonkhip as hip  # noqa: E402

hip.init(0)
ndev = hip.device_count()
n = 1 << 22
rng = np.random.default_rng(4242)
kg = np.array([[1, 2, 0], [68, 74, 0], [26, 45, 0], [65, 98, 0]], np.uint8)
pts = kg[rng.integers(0, 4, n)].reshape(-1)
sc = rng.integers(0, 17, n, dtype=np.uint8)
out = {"points": n, "devices_visible": ndev}
want = None
try:
    for ids in ([0], list(range(ndev))):
        hip.init_devices(ids)
        got = hip.msm_g1(pts, sc)
        want = want or got
        ok = got == want
        cached, fresh = [], []
        for _ in range(3):
            t0 = time.perf_counter()
            for _ in range(5):
                ok &= hip.msm_g1(pts, sc) == want
            cached.append((time.perf_counter() - t0) / 5 * 1e6)
            copies = [pts.copy() for _ in range(3)]
            t0 = time.perf_counter()
            for c in copies:
                ok &= hip.msm_g1(c, sc) == want
            fresh.append((time.perf_counter() - t0) / 3 * 1e6)
        cached.sort()
        fresh.sort()
        out["devices_" + "_".join(map(str, ids))] = {
            "srs_cached_us": round(cached[0], 1), "srs_cached_median_us": round(cached[1], 1),
            "srs_uploaded_us": round(fresh[0], 1), "srs_uploaded_median_us": round(fresh[1], 1),
            "same_result": bool(ok)}
finally:
    hip.init_devices([0])
print(json.dumps(out), flush=True)
