#!/bin/bash
# round-6 batch 6: the new seeded random-shape poly_mul parity test, smoke(), and the default bench
# line twice (box variance of the C5 and C3 components)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r6
mkdir -p $O
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_polymul_gpu.py -k "random or batch" \
    > $O/b6_tests.txt 2>&1 || { tail -40 $O/b6_tests.txt; exit 1; }
tail -3 $O/b6_tests.txt
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/b6_smoke.txt 2>&1 || { cat $O/b6_smoke.txt; exit 1; }
tail -1 $O/b6_smoke.txt
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $O/b6_bench$i.json 2> $O/b6_bench$i.err || { tail $O/b6_bench$i.err; exit 1; }
  python3 - $O/b6_bench$i.json <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
c = d["components"]
p, q = c["prove_2^20_gates"], c["prove_2^20_gates_preprocessed"]
print(d["value"], d["roofline"]["frac"], "prove", p["median_ms"], p["best_ms"], p["roofline"]["frac"], "pre", q["median_ms"],
      "ntt29", c["ntt29_2^20_forward"]["ms"], "pmul", c["poly_mul_2^19x2^19"]["ms"], "toy", c["cpu_reference_other"]["toy_prove_4_gates"]["dropin_us"])
PY
done
