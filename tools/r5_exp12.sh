#!/bin/bash
# round-5 batch 12: the full GPU suite on the new defaults (DBUF13, SWZ12 = 4); the standalone lo = 0
# passes with the pass-wide swizzle and set-based barriers (build/var/lib_louswz.so); the pass kernels
# with buffers alternating across a block's arrays, no barrier between arrays (build/var/lib_alt.so):
# their tests, then C3 and prove A/B
set -u
export TMPDIR=/tmp
O=gpurun_out/r5e12
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu tests > $O/tests.log 2>&1 || { echo "tests failed"; tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
PLK_LIB=$PWD/plonk.c_amd/build/var/lib_louswz.so timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_ntt_gpu.py tests/test_polymul_gpu.py > $O/lo_tests.log 2>&1 || { echo "louswz tests failed"; tail -30 $O/lo_tests.log; exit 1; }
tail -1 $O/lo_tests.log
PLK_LIB=$PWD/plonk.c_amd/build/var/lib_alt.so timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_ntt_gpu.py tests/test_polymul_gpu.py tests/test_prove_gpu.py > $O/alt_tests.log 2>&1 || { echo "alt tests failed"; tail -30 $O/alt_tests.log; exit 1; }
tail -1 $O/alt_tests.log
timeout -k 10 300 bash tools/c3_lib_ab.sh 3 > $O/c3ab.txt 2>&1 || { echo "c3 ab failed"; cat $O/c3ab.txt; exit 1; }
cat $O/c3ab.txt
LIBS="plonk.c_amd/libplonkhip.so plonk.c_amd/build/var/lib_alt.so" timeout -k 10 500 bash tools/prove_lib_ab.sh 4 > $O/prove_ab.txt 2>&1 || { echo "prove ab failed"; tail $O/prove_ab.txt; exit 1; }
cat $O/prove_ab.txt
echo done
