#!/bin/bash
# round-5 batch 33: graph setup failures fall back to direct launches -- the prover tests
set -u
export TMPDIR=/tmp
O=gpurun_out/r5e33
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_prove_gpu.py tests/test_prove_helpers_gpu.py > $O/tests.log 2>&1 || { echo "tests failed"; tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
echo done
