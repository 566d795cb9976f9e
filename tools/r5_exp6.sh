#!/bin/bash
# round-5 batch 6: a standalone transform's lo = 0 pass at 512 threads x 8 elements (build/var/lib_lor3.so):
# its NTT tests, then C3 timings alternating with the default build; the inverse passes' mod-17
# output as arithmetic (build/var/lib_m17a.so) against the LDS table, per kernel, three alternations
set -u
export TMPDIR=/tmp
O=gpurun_out/r5e6
mkdir -p $O
PLK_LIB=$PWD/plonk.c_amd/build/var/lib_lor3.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_ntt_gpu.py tests/test_polymul_gpu.py > $O/lor3_tests.log 2>&1 || { echo "lor3 tests failed"; tail -30 $O/lor3_tests.log; exit 1; }
tail -1 $O/lor3_tests.log
LIBS="plonk.c_amd/libplonkhip.so plonk.c_amd/build/var/lib_lor3.so" timeout -k 10 300 tools/c3_lib_ab.sh 4 > $O/c3ab.txt 2>&1 || { echo "c3 ab failed"; cat $O/c3ab.txt; exit 1; }
cat $O/c3ab.txt
for r in 1 2 3; do
  AB_KSUB=wt_inv timeout -k 10 400 tools/ab_kernels.sh >> $O/m17.txt 2>&1 || { echo "ab kernels failed"; tail $O/m17.txt; exit 1; }
done
cat $O/m17.txt
echo done
