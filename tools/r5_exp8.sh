#!/bin/bash
# round-5 batch 8: the 2^13 centre with swizzled exchanges (build/var/lib_swz1.so: everywhere
# conflict-free; lib_swz2.so: only where the padded layout conflicts) against the padded default --
# prover tests on swz1, then prove wall time alternating and the centre per kernel
set -u
export TMPDIR=/tmp
O=gpurun_out/r5e8
mkdir -p $O
PLK_LIB=$PWD/plonk.c_amd/build/var/lib_swz1.so timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_prove_gpu.py > $O/swz1_tests.log 2>&1 || { echo "swz1 tests failed"; tail -30 $O/swz1_tests.log; exit 1; }
tail -1 $O/swz1_tests.log
timeout -k 10 500 bash tools/prove_lib_ab.sh 3 > $O/prove_ab.txt 2>&1 || { echo "prove ab failed"; tail $O/prove_ab.txt; exit 1; }
cat $O/prove_ab.txt
for r in 1 2; do
  AB_KSUB=wt_center timeout -k 10 400 bash tools/ab_kernels.sh >> $O/center.txt 2>&1 || { echo "ab kernels failed"; tail $O/center.txt; exit 1; }
done
cat $O/center.txt
echo done
