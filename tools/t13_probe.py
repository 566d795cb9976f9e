#!/usr/bin/env python3
"""Plans with 2^12 tiles where the defaults use 2^13 (PLK_OPT_NTT_T13_MIN_K, set before plk_init):
standalone F29 / BabyBear transforms and poly_mul products of 2^21.. points against independent
references (diagnostic).   python3 tools/t13_probe.py <T13_MIN_K> [k ...]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in ("plonk.c_amd", "oracle", "tests", os.path.join("tests", "golden")):
    sys.path.insert(0, os.path.join(ROOT, p))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import gen  # noqa: E402
import plonkhip as hip  # noqa: E402
from pyoracle import Oracle  # noqa: E402
from test_ntt_gpu import P, P29, ntt_dif_reference  # noqa: E402

hip.set_option("NTT_T13_MIN_K", int(sys.argv[1]))
hip.init(0)
orc = Oracle()
ks = [int(x) for x in sys.argv[2:]] or [21, 22]
st = torch.cuda.current_stream()
for k in ks:
    for name, p, g, fn in (("f29", P29, 3, hip.ntt29_dev), ("bb", P, 31, hip.ntt_dev)):
        x = np.random.default_rng(k).integers(0, p, 1 << k, dtype=np.int64)
        d = torch.from_numpy(x.astype(np.int32)).cuda()
        fn(d, k, False, st)
        torch.cuda.synchronize()
        got = d.cpu().numpy().view(np.uint32).astype(np.uint64)
        ok_f = bool(np.array_equal(got, ntt_dif_reference(x, k, p, g))) if k <= 23 else None
        fn(d, k, True, st)
        torch.cuda.synchronize()
        back = d.cpu().numpy().view(np.uint32).astype(np.uint64)
        ok_i = bool(np.array_equal(back, (x.astype(np.uint64) * np.uint64(pow(2, k, p))) % np.uint64(p)))
        print("ntt %s 2^%d forward %s inverse %s" % (name, k, ok_f, ok_i), flush=True)
    la = (1 << (k - 1)) - 3
    a, b = gen.poly_inputs(k, la, la + 5)
    got = hip.poly_mul(a, b)
    print("poly_mul %d x %d (2^%d) %s" % (la, la + 5, k, got == orc.poly_mul_ntt(a, b)), flush=True)
