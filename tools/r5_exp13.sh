#!/bin/bash
# round-5 batch 13: the 2^13 centre at 512 threads x 16 registers (build/var/lib_rc4.so: 3 exchanges per
# transform, 5 barriers per item under the set rules) against 1024 x 8 -- prover tests, prove A/B, per kernel
set -u
export TMPDIR=/tmp
O=gpurun_out/r5e13
mkdir -p $O
PLK_LIB=$PWD/plonk.c_amd/build/var/lib_rc4.so timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_prove_gpu.py tests/test_polymul_gpu.py > $O/rc4_tests.log 2>&1 || { echo "rc4 tests failed"; tail -30 $O/rc4_tests.log; exit 1; }
tail -1 $O/rc4_tests.log
timeout -k 10 500 bash tools/prove_lib_ab.sh 3 > $O/prove_ab.txt 2>&1 || { echo "prove ab failed"; tail $O/prove_ab.txt; exit 1; }
cat $O/prove_ab.txt
echo done
