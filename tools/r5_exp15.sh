#!/bin/bash
# round-5 batch 15: C3's 2^12 kernels -- the high passes with a third exchange buffer so their wave-local
# exchange skips its barrier (build/var/lib_tri.so), plus the centre's b pass in a buffer of its own
# (lib_tri2b.so): tests on lib_tri2b.so, then C3 A/B alternating against the default build
set -u
export TMPDIR=/tmp
O=gpurun_out/r5e15
mkdir -p $O
PLK_LIB=$PWD/plonk.c_amd/build/var/lib_tri2b.so timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_ntt_gpu.py tests/test_polymul_gpu.py tests/test_prove_gpu.py > $O/tests.log 2>&1 || { echo "tri2b tests failed"; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 400 bash tools/c3_lib_ab.sh 4 > $O/c3ab.txt 2>&1 || { echo "c3 ab failed"; cat $O/c3ab.txt; exit 1; }
cat $O/c3ab.txt
echo done
