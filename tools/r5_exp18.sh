#!/bin/bash
# round-5 batch 18: the 2^12 centre loading its twiddle table after the first item's operand loads
# (build/var/lib_latetw.so: both latencies overlap) -- product tests, then C3 A/B alternating
set -u
export TMPDIR=/tmp
O=gpurun_out/r5e18
mkdir -p $O
PLK_LIB=$PWD/plonk.c_amd/build/var/lib_latetw.so timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_polymul_gpu.py tests/test_prove_gpu.py > $O/tests.log 2>&1 || { echo "latetw tests failed"; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 400 bash tools/c3_lib_ab.sh 4 > $O/c3ab.txt 2>&1 || { echo "c3 ab failed"; cat $O/c3ab.txt; exit 1; }
cat $O/c3ab.txt
echo done
