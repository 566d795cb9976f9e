#!/usr/bin/env python3
"""Quick device-time check of the NTT / poly_mul kernels (tuning aid)."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "plonk.c_amd"))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import plonkhip as hip  # noqa: E402
from bench import event_avg_ms  # noqa: E402

hip.tune_from_env()   # PLK_TUNE="NAME=value,..." (plk_set_option), tuning runs only
hip.init(0)
PLAN = sys.argv[sys.argv.index("--plan") + 1] if "--plan" in sys.argv else None
if PLAN:   # every NTT pass launch of this run, in order (tools/ntt_roofline.py --plan)
    hip.set_option("NTT_LAUNCH_LOG", 1)
dev = torch.device("cuda", 0)
st = torch.cuda.current_stream()
out = {}
quick = "--quick" in sys.argv
for k in ((20, 22) if quick else (16, 20, 22, 23)):
    bufs = [torch.randint(0, 2013265921, (1 << k,), dtype=torch.int64, device=dev).to(torch.int32) for _ in range(4)]
    avg, med = event_avg_ms(torch, st, lambda i: hip.ntt_dev(bufs[i % 4], k, False, st), 40)
    out["ntt_fwd_2^%d_us" % k] = round(avg * 1e3, 2)
    out["ntt_fwd_2^%d_Gelem_s" % k] = round((1 << k) / (avg * 1e-3) / 1e9, 1)
for k in ((20,) if quick else (20, 22)):
    nb = 8
    bb_ = [torch.randint(0, 2013265921, (nb, 1 << k), dtype=torch.int64, device=dev).to(torch.int32) for _ in range(2)]
    avg, med = event_avg_ms(torch, st, lambda i: hip.ntt_batch_dev(bb_[i % 2], k, nb, False, st), 20)
    out["ntt_fwd_2^%d_batch8_us" % k] = round(avg * 1e3, 2)
    out["ntt_fwd_2^%d_batch8_Gelem_s" % k] = round(nb * (1 << k) / (avg * 1e-3) / 1e9, 1)
P29 = 7 * (1 << 26) + 1
for k in ((20, 22) if quick else (16, 20, 22, 23)):
    bufs = [torch.randint(0, P29, (1 << k,), dtype=torch.int64, device=dev).to(torch.int32) for _ in range(4)]
    avg, med = event_avg_ms(torch, st, lambda i: hip.ntt29_dev(bufs[i % 4], k, False, st), 40)
    out["ntt29_fwd_2^%d_us" % k] = round(avg * 1e3, 2)
    out["ntt29_fwd_2^%d_Gelem_s" % k] = round((1 << k) / (avg * 1e-3) / 1e9, 1)
for k in ((20,) if quick else (20, 22)):
    nb = 8
    bb_ = [torch.randint(0, P29, (nb, 1 << k), dtype=torch.int64, device=dev).to(torch.int32) for _ in range(2)]
    avg, med = event_avg_ms(torch, st, lambda i: hip.ntt29_batch_dev(bb_[i % 2], k, nb, False, st), 20)
    out["ntt29_fwd_2^%d_batch8_us" % k] = round(avg * 1e3, 2)
    out["ntt29_fwd_2^%d_batch8_Gelem_s" % k] = round(nb * (1 << k) / (avg * 1e-3) / 1e9, 1)
for la, lb in (((1 << 19, 1 << 19),) if quick else
               ((1 << 12, 1 << 12), (1 << 16, 1 << 16), (1 << 19, 1 << 19), (3 * (1 << 20) + 4, (1 << 20) + 3))):
    a = torch.randint(0, 17, (la,), dtype=torch.int16, device=dev).to(torch.uint8)
    b = torch.randint(0, 17, (lb,), dtype=torch.int16, device=dev).to(torch.uint8)
    o = torch.zeros(la + lb - 1, dtype=torch.uint8, device=dev)
    nz = torch.zeros(4, dtype=torch.int32, device=dev)
    work = torch.zeros(max(4, hip.poly_mul_workspace(la, lb)), dtype=torch.uint8, device=dev)
    avg, med = event_avg_ms(torch, st, lambda i: hip.poly_mul_dev(a, la, b, lb, o, nz, work, st), 20)
    out["poly_mul_%dx%d_us" % (la, lb)] = round(avg * 1e3, 2)
print(json.dumps(out))
if PLAN:
    with open(PLAN, "w") as f:
        json.dump({"launches": hip.ntt_launch_log(1 << 16)}, f)
