#!/bin/bash
# round-5 batch 34: A2 B2's shifted bytes from the neighbour lane (DPP row_shr:1) in the derived
# first pass -- its parity tests, then prove A/B against the build that loads them
# (build/var/lib_nodpp.so), 31 calls per median
set -u
export TMPDIR=/tmp
O=gpurun_out/r5e34
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_prove_gpu.py -k "derive or golden or tiles13 or sweep or graph" > $O/tests.log 2>&1 || { echo "tests failed"; tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
PROVE_REPS=31 timeout -k 10 900 tools/prove_lib_ab.sh 5 > $O/prove_ab.txt 2>&1 || { echo "prove ab failed"; tail $O/prove_ab.txt; exit 1; }
cat $O/prove_ab.txt
echo done
