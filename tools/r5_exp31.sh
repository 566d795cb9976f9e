#!/bin/bash
# round-5 batch 31: the poly_mul option sweep
set -u
export TMPDIR=/tmp
O=gpurun_out/r5e31
mkdir -p $O
timeout -k 10 500 python -u -m pytest -x -q --timeout 400 --timeout-method thread -m gpu tests/test_polymul_gpu.py -k "option_sweep" > $O/tests.log 2>&1 || { echo "tests failed"; tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
echo done
