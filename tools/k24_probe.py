#!/usr/bin/env python3
"""Probe (tuning aid): 2^24-point poly_mul products (three-pass plans) through the device API,
timed and checked against the oracle; prints as it goes."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "plonk.c_amd"), os.path.join(ROOT, "tests", "golden"), os.path.join(ROOT, "oracle")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

import gen  # noqa: E402
from pyoracle import Oracle  # noqa: E402

# PLK_LIB: any build (older ones lack later symbols: bind the two used here directly)
import ctypes as C  # noqa: E402
L = C.CDLL(os.environ.get("PLK_LIB") or os.path.join(ROOT, "plonk.c_amd", "libplonkhip.so"))
L.plk_init.argtypes = [C.c_int]
L.plk_poly_mul_workspace.restype = C.c_size_t
L.plk_poly_mul_workspace.argtypes = [C.c_size_t, C.c_size_t]
L.plk_poly_mul_dev.argtypes = [C.c_void_p, C.c_size_t, C.c_void_p, C.c_size_t, C.c_void_p, C.c_void_p,
                               C.c_void_p, C.c_void_p]
assert L.plk_init(0) == 0
o = Oracle()
dev = torch.device("cuda", 0)
for la, lb in [(5000000, 3600000), (5000000, 3800000)]:
    a, b = gen.poly_inputs(la * 31 + lb, la, lb)
    da, db = torch.from_numpy(a).to(dev), torch.from_numpy(b).to(dev)
    out = torch.zeros(la + lb - 1, dtype=torch.uint8, device=dev)
    nz = torch.zeros(4, dtype=torch.int32, device=dev)
    work = torch.zeros(max(L.plk_poly_mul_workspace(la, lb), 4), dtype=torch.uint8, device=dev)
    torch.cuda.synchronize()
    t = time.time()
    rc = L.plk_poly_mul_dev(da.data_ptr(), la, db.data_ptr(), lb, out.data_ptr(), nz.data_ptr(), work.data_ptr(),
                            C.c_void_p(torch.cuda.current_stream().cuda_stream))
    assert rc == 0, rc
    torch.cuda.synchronize()
    print("gpu", la, lb, "%.3f s" % (time.time() - t), flush=True)
    n = int(nz[0].item()) or 1
    ok = bytes(out[:n].cpu().numpy()) == o.poly_mul_ntt(a, b)
    print("parity", la, lb, ok, flush=True)
