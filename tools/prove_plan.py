#!/usr/bin/env python3
"""The NTT pass launch plan of ONE 2^k-gate proof (plk_ntt_launch_log), for the offline roofline
tools: rocprof records each launch's grid, not how many arrays a table pass's blocks walk or how
many pass units the persistent center kernel runs.  Usage:
    python tools/prove_plan.py [--pre] [k] > plan.json"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "plonk.c_amd"), os.path.join(ROOT, "tests", "golden")]
import torch  # noqa: E402

import gen  # noqa: E402
import plonkhip as hip  # noqa: E402

hip.tune_from_env()
hip.init(0)
pre = "--pre" in sys.argv
k = int(([a for a in sys.argv[1:] if a != "--pre"] or ["20"])[0])
n = 1 << k
hpolys, chal, rnd, zh, pts = gen.prove_instance(n, 51, 2 * n + 8)
polys = [torch.from_numpy(p).to("cuda") for p in hpolys]
pr = hip.Prover(n, zh, pts)
if pre:
    pr.preprocess(polys)
pr.rounds_dev(polys, chal, rnd, preprocessed=pre)
hip.ntt_launch_log()                      # (drop anything before the recorded proof)
hip.set_option("NTT_LAUNCH_LOG", 1)
pr.rounds_dev(polys, chal, rnd, preprocessed=pre)
hip.set_option("NTT_LAUNCH_LOG", 0)
print(json.dumps({"k": k, "preprocessed": pre, "launches": hip.ntt_launch_log()}))
