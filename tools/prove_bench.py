#!/usr/bin/env python3
"""Prove-shaped pipeline timing at n = 2^k gates (tuning aid; run under rocprofv3 for the
per-kernel split).  Usage: python tools/prove_bench.py [--pre] [k ...]"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "plonk.c_amd"))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import plonkhip as hip  # noqa: E402
from bench import prove_component  # noqa: E402

hip.tune_from_env()   # PLK_TUNE="NAME=value,..." (plk_set_option), tuning runs only
hip.init(0)
dev = torch.device("cuda", 0)
pre = "--pre" in sys.argv   # the preprocessed-circuit path (plk_prover_preprocess) instead
ks = [int(x) for x in sys.argv[1:] if x != "--pre"] or [16, 18, 20]
reps = int(os.environ.get("PROVE_REPS", "9"))   # calls per median
print(json.dumps({"prove_2^%d" % k: prove_component(torch, hip, dev, k, reps=reps, preprocessed=pre) for k in ks}))
