#!/bin/bash
# round-5 batch 29: the option sweep at 2^20 against the golden proof
set -u
export TMPDIR=/tmp
O=gpurun_out/r5e29
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_prove_gpu.py -k "sweep" > $O/tests.log 2>&1 || { echo "tests failed"; tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
echo done
