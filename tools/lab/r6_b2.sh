#!/bin/bash
# round-6 batch 2: the prover's profile / launch-count entry points, the drop-in at both small-size
# policies (toy calls on the host / every call on the GPU), and the bench line's C5 roofline
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r6
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
    tests/test_prove_gpu.py -k "profile or launches or 2_20_vs_golden" tests/test_dropin_gpu.py tests/test_reference_suite.py \
    > gpurun_out/r6/b2_tests.txt 2>&1 || { tail -60 gpurun_out/r6/b2_tests.txt; exit 1; }
tail -3 gpurun_out/r6/b2_tests.txt
timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --components prove,cpu > gpurun_out/r6/b2_bench.json 2> gpurun_out/r6/b2_bench.err \
    || { tail -30 gpurun_out/r6/b2_bench.err; exit 1; }
python3 - <<'PY'
import json
d = json.load(open("gpurun_out/r6/b2_bench.json"))
c = d["components"]
for k in ("prove_2^20_gates", "prove_2^20_gates_preprocessed"):
    v = c[k]
    print(k, v["median_ms"], v["launches"], json.dumps(v["roofline"])[:900])
print(json.dumps(c["cpu_reference_other"]["toy_prove_4_gates"]))
PY
