#!/usr/bin/env python3
"""Config C3's two shapes alone, for counter passes (tuning aid): the single 2^20 forward
transform over F29 (plk_ntt29_dev) and poly_mul 2^19 x 2^19 (plk_poly_mul_dev), REPS launches
each, back to back on one stream.   python tools/c3_bench.py [reps]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "plonk.c_amd"))
import torch  # noqa: E402

import plonkhip as hip  # noqa: E402

hip.tune_from_env()
hip.init(0)
reps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
dev = torch.device("cuda", 0)
st = torch.cuda.current_stream()
P29 = 7 * (1 << 26) + 1
bufs = [torch.randint(0, P29, (1 << 20,), dtype=torch.int64, device=dev).to(torch.int32) for _ in range(4)]
for i in range(reps):
    hip.ntt29_dev(bufs[i % 4], 20, False, st)
la = lb = 1 << 19
a = torch.randint(0, 17, (la,), dtype=torch.int16, device=dev).to(torch.uint8)
b = torch.randint(0, 17, (lb,), dtype=torch.int16, device=dev).to(torch.uint8)
o = torch.zeros(la + lb - 1, dtype=torch.uint8, device=dev)
nz = torch.zeros(4, dtype=torch.int32, device=dev)
work = torch.zeros(hip.poly_mul_workspace(la, lb), dtype=torch.uint8, device=dev)
for i in range(reps):
    hip.poly_mul_dev(a, la, b, lb, o, nz, work, st)
torch.cuda.synchronize()
print("c3 done")
