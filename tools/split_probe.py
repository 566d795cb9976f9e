#!/usr/bin/env python3
"""What a strong-scaled proof could gain (lab tool): device time of the prover's
round-3 product batches split into fewer products per GPU.  At n = 2^20 gates the 2^21 batch
holds 10 products of ~(n+2) x (n+3) coefficients and the 2^22 batch 3 of ~(2n+5) x (2n+5); a
strong-scaled proof would run k of them per GPU.  Times batches of k = 1 .. all products
(distinct random operands, bytes in / bytes out, plk_poly_mul_batch_dev) with an event pair
around `reps` back-to-back calls, and prints one JSON line per (size, k).

    python tools/split_probe.py [reps]
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "plonk.c_amd"))


def main():
    import torch

    import plonkhip as hip
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 10
    hip.init(0)
    dev = torch.device("cuda", 0)
    st = torch.cuda.current_stream()
    n = 1 << 20
    g = torch.Generator(device=dev).manual_seed(7)
    for (la, lb, total) in ((n + 2, n + 3, 10), (2 * n + 5, 2 * n + 5, 3)):
        a = [torch.randint(0, 17, (la,), generator=g, device=dev, dtype=torch.int16).to(torch.uint8)
             for _ in range(total)]
        b = [torch.randint(0, 17, (lb,), generator=g, device=dev, dtype=torch.int16).to(torch.uint8)
             for _ in range(total)]
        out = [torch.empty(la + lb - 1 + 64, dtype=torch.uint8, device=dev) for _ in range(total)]
        for k in range(1, total + 1):
            jobs = [(a[i], la, b[i], lb, out[i], 0) for i in range(k)]
            wb = hip.poly_mul_batch_workspace(jobs)
            work = torch.empty(max(wb, 1), dtype=torch.uint8, device=dev)
            hip.poly_mul_batch_dev(jobs, work, wb, st)       # warm
            torch.cuda.synchronize()
            best = None
            for _ in range(3):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                hip.poly_mul_batch_dev(jobs, work, wb, st)
                e0.record(st)
                for _ in range(reps):
                    hip.poly_mul_batch_dev(jobs, work, wb, st)
                e1.record(st)
                torch.cuda.synchronize()
                ms = e0.elapsed_time(e1) / reps
                best = ms if best is None else min(best, ms)
            print(json.dumps({"la": la, "lb": lb, "products": k, "of": total, "us": round(best * 1e3, 1)}),
                  flush=True)


if __name__ == "__main__":
    main()
