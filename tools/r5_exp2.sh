#!/bin/bash
# round-5 batch 2: prover GPU tests with round 4's chunk aggregates (PROVE_EVAL_AGG), its A/B, C3 counters
set -u
export TMPDIR=/tmp
O=gpurun_out/r5e2
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_prove_gpu.py tests/test_prove_split_gpu.py tests/test_prove_helpers_gpu.py tests/test_dropin_gpu.py > $O/tests.log 2>&1 || { echo "tests failed"; tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 500 tools/prove_tune_ab.sh "PROVE_EVAL_AGG=0" "PROVE_EVAL_AGG=1" 3 > $O/ab.txt 2>&1 || { echo "ab failed"; tail $O/ab.txt; exit 1; }
cat $O/ab.txt
timeout -k 10 500 tools/c3_pmc.sh > $O/c3.log 2>&1 || { echo "c3 failed"; tail $O/c3.log; exit 1; }
echo done
