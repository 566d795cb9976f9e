#!/bin/bash
# round-5 final check: the whole GPU suite and the default bench line
set -u
export TMPDIR=/tmp
O=gpurun_out/r5final
mkdir -p $O
timeout -k 10 900 python -u -m pytest -q --timeout 400 --timeout-method thread -m gpu tests > $O/gpu_tests.log 2>&1 || { echo "gpu tests failed"; tail -40 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail $O/bench.err; exit 1; }
grep '^{' $O/bench.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['unit'], d['roofline']['frac'], d['components']['prove_2^20_gates']['median_ms'], d['components']['prove_2^20_gates_preprocessed']['median_ms'])"
echo done
