"""plk_msm_g1 over every visible GPU (plk_init_devices with distinct device ids): the multi-device
host-buffer path of srs_eval_at_s at 2^22 points, against device 0 alone; and one 2^20-gate proof
split over 2 and 3 distinct GPUs from C (plk_prover_attach_helpers: t_3 / t_2 and t_3 on helper
GPUs, products peer-copied back), inputs on device 0 (rounds_dev: the helpers copy the 7 inputs
they read) or already on every device (rounds_multi_dev), against the single-GPU proof and the
recorded answer.  Run by bench.py as a child process (its own contexts, a time limit) on multi-GPU
nodes; prints one JSON object."""
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


def split_prove(out, reps=7):
    import torch
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests", "golden"))
    import gen
    with open(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests", "golden",
                           "prove_2_20.json")) as f:
        g = json.load(f)
    n = g["n"]
    polys, chal, rnd, zh, pts_ = gen.prove_instance(n, g["seed"], g["srs_len"])
    sets = [[torch.from_numpy(p).to("cuda:%d" % d) for p in polys] for d in range(min(ndev, 3))]
    torch.cuda.set_device(0)

    def timed(fn):
        fn()
        t = []
        for _ in range(reps):
            t0 = time.perf_counter()
            r = fn()
            t.append(time.perf_counter() - t0)
        t.sort()
        return r, round(t[len(t) // 2] * 1e3, 3), round(t[0] * 1e3, 3)

    pr = hip.Prover(n, zh, pts_)
    single, ms, best = timed(lambda: pr.rounds_dev(sets[0], chal, rnd))
    res = {"single_gpu_median_ms": ms, "single_gpu_best_ms": best, "single_matches_golden": single.hex() == g["proof"]}
    for k in (1, 2):
        if ndev < 1 + k:
            break
        hip.init_devices(list(range(1 + k)))
        pr.attach_helpers(k)
        got, ms, best = timed(lambda: pr.rounds_dev(sets[0], chal, rnd))
        got2, ms2, best2 = timed(lambda: pr.rounds_multi_dev(sets[:1 + k], chal, rnd))
        res["gpus_%d" % (1 + k)] = {"inputs_on_device0_median_ms": ms, "inputs_on_device0_best_ms": best,
                                    "inputs_resident_median_ms": ms2, "inputs_resident_best_ms": best2,
                                    "matches_golden": got.hex() == g["proof"] and got2.hex() == g["proof"]}
        pr.attach_helpers(0)
    hip.init_devices([0])
    pr.close()
    out["prove_2^20_split_from_c"] = res


if ndev > 1:
    try:
        split_prove(out)
    except Exception as e:   # (reported in the line, never costs the MSM numbers above)
        out["prove_2^20_split_from_c"] = {"error": repr(e)[:300]}
print(json.dumps(out), flush=True)
