#!/bin/bash
# round-6 final check on the committed tree: the whole GPU suite, smoke(), the default bench line
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r6
mkdir -p $O
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest -q --timeout 300 --timeout-method thread -m gpu tests > $O/final_gpu_suite.txt 2>&1 \
    || { tail -30 $O/final_gpu_suite.txt; exit 1; }
tail -1 $O/final_gpu_suite.txt
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/final_smoke.txt 2>&1 || { cat $O/final_smoke.txt; exit 1; }
tail -1 $O/final_smoke.txt
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $O/final_bench.json 2> $O/final_bench.err || { tail $O/final_bench.err; exit 1; }
python3 - $O/final_bench.json <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
c = d["components"]
p = c["prove_2^20_gates"]
print(d["value"], d["roofline"]["frac"], d["checks"], "prove", p["median_ms"], p["launches"], p["roofline"]["frac"],
      "toy", c["cpu_reference_other"]["toy_prove_4_gates"]["dropin_us"], c["cpu_reference_other"]["toy_prove_4_gates"]["reference_cpu_us"])
PY
