#!/bin/bash
# round-5 batch 10: centre exchanges with one (padded) layout and barriers only where a wave's
# element set changes (PLK_NTT_CENTER_SWZ(12) = 3; build/var/lib_uni13.so: the 2^13 centre and the
# shared-operand pass, lib_uni.so: also the 2^12 centre) -- prover and product tests on lib_uni.so,
# then prove / C3 A/B alternating against the default build, and the centre per kernel
set -u
export TMPDIR=/tmp
O=gpurun_out/r5e10
mkdir -p $O
PLK_LIB=$PWD/plonk.c_amd/build/var/lib_uni.so timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_prove_gpu.py tests/test_polymul_gpu.py tests/test_ntt_gpu.py tests/test_prove_split_gpu.py > $O/uni_tests.log 2>&1 || { echo "uni tests failed"; tail -30 $O/uni_tests.log; exit 1; }
tail -1 $O/uni_tests.log
timeout -k 10 500 bash tools/prove_lib_ab.sh 3 > $O/prove_ab.txt 2>&1 || { echo "prove ab failed"; tail $O/prove_ab.txt; exit 1; }
cat $O/prove_ab.txt
timeout -k 10 300 bash tools/c3_lib_ab.sh 3 > $O/c3ab.txt 2>&1 || { echo "c3 ab failed"; cat $O/c3ab.txt; exit 1; }
cat $O/c3ab.txt
AB_KSUB=wt_ timeout -k 10 400 bash tools/ab_kernels.sh > $O/kern.txt 2>&1 || { echo "ab kernels failed"; tail $O/kern.txt; exit 1; }
cat $O/kern.txt
echo done
