#!/usr/bin/env python3
"""Config C3's shapes timed as bench.py times them (graph-replayed launches, tuning aid): the 2^20
forward transform over F29 and BabyBear, 8 per launch, and poly_mul 2^19 x 2^19 (one JSON line)."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "plonk.c_amd"))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import plonkhip as hip  # noqa: E402
from bench import graph_avg_ms  # noqa: E402

hip.tune_from_env()
hip.init(0)
dev = torch.device("cuda", 0)
torch.manual_seed(1)
out = {}
P29 = 7 * (1 << 26) + 1
b29 = [torch.randint(0, P29, (1 << 20,), dtype=torch.int64, device=dev).to(torch.int32) for _ in range(4)]
out["ntt29_2^20_us"] = round(graph_avg_ms(torch, lambda i, s: hip.ntt29_dev(b29[i % 4], 20, False, s), 50)[0] * 1e3, 2)
bb = [torch.randint(0, 2013265921, (1 << 20,), dtype=torch.int64, device=dev).to(torch.int32) for _ in range(4)]
out["ntt_bb_2^20_us"] = round(graph_avg_ms(torch, lambda i, s: hip.ntt_dev(bb[i % 4], 20, False, s), 50)[0] * 1e3, 2)
la = lb = 1 << 19
a = torch.randint(0, 17, (la,), dtype=torch.int16, device=dev).to(torch.uint8)
b = torch.randint(0, 17, (lb,), dtype=torch.int16, device=dev).to(torch.uint8)
o = torch.zeros(la + lb - 1, dtype=torch.uint8, device=dev)
nz = torch.zeros(4, dtype=torch.int32, device=dev)
work = torch.zeros(hip.poly_mul_workspace(la, lb), dtype=torch.uint8, device=dev)
hip.poly_mul_dev(a, la, b, lb, o, nz, work, torch.cuda.current_stream())
torch.cuda.synchronize()
ref = o.clone()
out["poly_mul_2^19_us"] = round(graph_avg_ms(torch, lambda i, s: hip.poly_mul_dev(a, la, b, lb, o, nz, work, s), 30)[0] * 1e3, 2)
torch.cuda.synchronize()
out["poly_mul_same_bytes"] = bool(torch.equal(o, ref))
import hashlib  # noqa: E402
out["poly_mul_sha"] = hashlib.sha256(o.cpu().numpy().tobytes()).hexdigest()[:12]
out["ntt29_sha"] = hashlib.sha256(b29[0].cpu().numpy().tobytes()).hexdigest()[:12]
print(json.dumps(out))
