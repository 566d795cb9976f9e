#!/bin/bash
# round-5 batch 24: A2 B2 in the t_2 product's first pass on 2^13 tiles only (the default now) --
# the whole GPU suite, C3 against the build without the derived branch, prove A/B modes 1 / 2
set -u
export TMPDIR=/tmp
O=gpurun_out/r5e24
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > $O/tests.log 2>&1 || { echo "tests failed"; tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
LIBS="plonk.c_amd/libplonkhip.so plonk.c_amd/build/var/lib_nodrv.so" timeout -k 10 300 tools/c3_lib_ab.sh 3 > $O/c3ab.txt 2>&1 || { echo "c3 ab failed"; cat $O/c3ab.txt; exit 1; }
cat $O/c3ab.txt
PROVE_REPS=31 timeout -k 10 900 tools/prove_opts_ab.sh 6 "PROVE_DERIVE_T2A=1" "PROVE_DERIVE_T2A=2" > $O/prove_ab.txt 2>&1 || { echo "prove ab failed"; tail $O/prove_ab.txt; exit 1; }
cat $O/prove_ab.txt
echo done
