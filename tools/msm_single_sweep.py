#!/usr/bin/env python3
"""One 2^22-point MSM per launch under one launch-geometry setting (tuning aid): run once per
setting in its own process (the PLK_MSM_* switches are read once), e.g.
    PLK_MSM_THREADS=256 python tools/msm_single_sweep.py
Prints the setting and bench.single_msm_component's numbers (graph-replayed, cold inputs)."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "plonk.c_amd"))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import plonkhip as hip  # noqa: E402
from bench import make_msm_sets, single_msm_component  # noqa: E402

hip.tune_from_env()   # PLK_TUNE="NAME=value,..." (plk_set_option), tuning runs only
hip.init(0)
dev = torch.device("cuda", 0)
n, sets = 1 << 22, 40
pts, sc = make_msm_sets(torch, n, sets, dev, 1234)
env = {k: v for k, v in os.environ.items() if k.startswith("PLK_MSM") or k == "PLK_TUNE"}
best = min((single_msm_component(torch, hip, pts, sc, n, sets, dev) for _ in range(3)),
           key=lambda c: c["device_us_per_msm"])
print(json.dumps({"env": env, "us": best["device_us_per_msm"], "median_us": best["median_us"], "frac": best["frac"]}))
