#!/bin/bash
# round-5 batch 32: re-check two pass-kernel switches on the final code -- the inverse passes'
# next-job prefetch (build/var/lib_pfi.so) and per-register buffer resources for byte loads
# (lib_krsrc.so): their NTT / poly_mul tests, prove A/B at 31 calls, C3 A/B
set -u
export TMPDIR=/tmp
O=gpurun_out/r5e32
mkdir -p $O
for v in pfi krsrc; do
  PLK_LIB=$PWD/plonk.c_amd/build/var/lib_$v.so timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_ntt_gpu.py tests/test_polymul_gpu.py tests/test_prove_gpu.py -k "not tile12 and not tiles13" > $O/tests_$v.log 2>&1 || { echo "$v tests failed"; tail -30 $O/tests_$v.log; exit 1; }
  tail -1 $O/tests_$v.log
done
PROVE_REPS=31 timeout -k 10 900 tools/prove_lib_ab.sh 4 > $O/prove_ab.txt 2>&1 || { echo "prove ab failed"; tail $O/prove_ab.txt; exit 1; }
cat $O/prove_ab.txt
timeout -k 10 400 tools/c3_lib_ab.sh 3 > $O/c3ab.txt 2>&1 || { echo "c3 ab failed"; cat $O/c3ab.txt; exit 1; }
cat $O/c3ab.txt
echo done
