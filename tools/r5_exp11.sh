#!/bin/bash
# round-5 batch 11: the full GPU suite on the new default (UNI 2^13 centre), the centres with one
# pass-wide conflict-free swizzle (build/var/lib_uswz.so), then the 2^13 high passes
# double-buffered (build/var/lib_dbuf13.so: one barrier per exchange) -- its prover tests, prove A/B
# alternating, per-kernel pass times
set -u
export TMPDIR=/tmp
O=gpurun_out/r5e11
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu tests > $O/tests.log 2>&1 || { echo "tests failed"; tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
PLK_LIB=$PWD/plonk.c_amd/build/var/lib_dbuf13.so timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_prove_gpu.py tests/test_polymul_gpu.py > $O/dbuf_tests.log 2>&1 || { echo "dbuf13 tests failed"; tail -30 $O/dbuf_tests.log; exit 1; }
tail -1 $O/dbuf_tests.log
PLK_LIB=$PWD/plonk.c_amd/build/var/lib_uswz.so timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_prove_gpu.py tests/test_polymul_gpu.py tests/test_ntt_gpu.py > $O/uswz_tests.log 2>&1 || { echo "uswz tests failed"; tail -30 $O/uswz_tests.log; exit 1; }
tail -1 $O/uswz_tests.log
timeout -k 10 300 bash tools/c3_lib_ab.sh 3 > $O/c3ab.txt 2>&1 || { echo "c3 ab failed"; cat $O/c3ab.txt; exit 1; }
cat $O/c3ab.txt
timeout -k 10 500 bash tools/prove_lib_ab.sh 3 > $O/prove_ab.txt 2>&1 || { echo "prove ab failed"; tail $O/prove_ab.txt; exit 1; }
cat $O/prove_ab.txt
AB_KSUB=wt_ timeout -k 10 400 bash tools/ab_kernels.sh > $O/kern.txt 2>&1 || { echo "ab kernels failed"; tail $O/kern.txt; exit 1; }
cat $O/kern.txt
echo done
