#!/usr/bin/env python3
"""Tuning sweep for the MSM kernel on one GPU (not part of the bench contract).

Times the 2^22-point MSM over rotated input sets (> 512 MiB, Infinity-Cache-cold) as
  eager   : one ctypes launch per MSM (host-launch bound)
  graph   : the same launches captured once in a HIP graph and replayed
  batchB  : plk_msm_g1_batch_dev, B MSMs per launch
and prints per-MSM device time, wall time and GB/s.  Block size via PLK_MSM_THREADS.
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "plonk.c_amd"))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import plonkhip as hip  # noqa: E402
from bench import make_msm_sets  # noqa: E402


def main():
    log2n = int(sys.argv[1]) if len(sys.argv) > 1 else 22
    n = 1 << log2n
    dev = torch.device("cuda", 0)
    hip.tune_from_env()   # PLK_TUNE="NAME=value,..." (plk_set_option), tuning runs only
    hip.init(0)
    st = torch.cuda.current_stream()
    sets = 40 if log2n >= 22 else 64
    pts, sc = make_msm_sets(torch, n, sets, dev, 5)
    K = 200
    res = torch.zeros((K, hip.MSM_RESULT_BYTES), dtype=torch.uint8, device=dev)
    out = {"log2n": log2n, "threads_env": os.environ.get("PLK_MSM_THREADS")}

    def timed(fn, reps=3):
        best = None
        for _ in range(reps):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            fn()
            torch.cuda.synchronize()
            dt = time.perf_counter() - t0
            best = dt if best is None else min(best, dt)
        return best

    def eager():
        for i in range(K):
            hip.msm_g1_dev(pts[i % sets], sc[i % sets], n, res[i], st)

    dt = timed(eager)
    out["eager_us_per_msm"] = round(dt / K * 1e6, 2)
    # graph
    gs = torch.cuda.Stream()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=gs):
        cs = torch.cuda.current_stream()
        for i in range(K):
            hip.msm_g1_dev(pts[i % sets], sc[i % sets], n, res[i], cs)
    dt = timed(lambda: g.replay())
    out["graph_us_per_msm"] = round(dt / K * 1e6, 2)
    out["graph_GBs"] = round(4 * n / (dt / K) / 1e9, 1)
    # batched
    for B in (1, 2, 4, 8, 20, 40):
        if sets % B:
            continue
        nl = K // B

        def batched():
            for j in range(nl):
                s0 = (j * B) % sets
                hip.msm_g1_batch_dev(pts[s0], 3 * n, sc[s0], n, n, B, res[j * B], st)
        dt = timed(batched)
        # device time per launch via events
        evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(nl)]
        for j in range(nl):
            s0 = (j * B) % sets
            evs[j][0].record(st)
            hip.msm_g1_batch_dev(pts[s0], 3 * n, sc[s0], n, n, B, res[j * B], st)
            evs[j][1].record(st)
        torch.cuda.synchronize()
        dev_ms = sorted(a.elapsed_time(b) for a, b in evs)
        avg = sum(dev_ms) / len(dev_ms)
        out["batch%d" % B] = {"wall_us_per_msm": round(dt / K * 1e6, 2),
                              "dev_us_per_launch": round(avg * 1e3, 2),
                              "dev_us_per_msm": round(avg * 1e3 / B, 2),
                              "GBs_dev": round(4 * n * B / (avg * 1e-3) / 1e9, 1)}
    # correctness spot check: every record agrees with a fresh single launch
    torch.cuda.synchronize()
    bad = int(res[:, hip.MSM_IRREGULAR_OFFSET:hip.MSM_IRREGULAR_OFFSET + 4].view(torch.int32).sum().item())
    r1 = torch.zeros((1, hip.MSM_RESULT_BYTES), dtype=torch.uint8, device=dev)
    hip.msm_g1_dev(pts[0], sc[0], n, r1[0], st)
    torch.cuda.synchronize()
    out["irregular"] = bad
    out["set0_g1"] = bytes(r1[0, hip.MSM_G1_OFFSET:hip.MSM_G1_OFFSET + 3].cpu().numpy()).hex()
    out["set0_batch_g1"] = bytes(res[0, hip.MSM_G1_OFFSET:hip.MSM_G1_OFFSET + 3].cpu().numpy()).hex()
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
