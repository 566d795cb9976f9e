#!/bin/bash
# round-5 batch 16: F29 centres reading {w, p - w} twiddle pairs (no subtraction in the forward DIF):
# build/var/lib_pw12.so the 2^12 centre (C3), lib_pw.so both (the 2^13 one with 2^11 pairs) -- tests on
# lib_pw.so, then C3 and prove A/B alternating against the default build
set -u
export TMPDIR=/tmp
O=gpurun_out/r5e16
mkdir -p $O
PLK_LIB=$PWD/plonk.c_amd/build/var/lib_pw.so timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_polymul_gpu.py tests/test_prove_gpu.py > $O/tests.log 2>&1 || { echo "pw tests failed"; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 400 bash tools/c3_lib_ab.sh 3 > $O/c3ab.txt 2>&1 || { echo "c3 ab failed"; cat $O/c3ab.txt; exit 1; }
cat $O/c3ab.txt
LIBS="plonk.c_amd/libplonkhip.so plonk.c_amd/build/var/lib_pw.so" timeout -k 10 500 bash tools/prove_lib_ab.sh 3 > $O/prove_ab.txt 2>&1 || { echo "prove ab failed"; tail $O/prove_ab.txt; exit 1; }
cat $O/prove_ab.txt
echo done
