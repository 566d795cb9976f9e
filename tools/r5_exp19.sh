#!/bin/bash
# round-5 batch 19: A2 B2 inside the t_2 product's first forward pass (PROVE_DERIVE_T2A = 2) --
# its parity tests, prove A/B against t2a_kernel (mode 1), and C3 against a build with the
# derived-operand branch compiled out (build/var/lib_nodrv.so: the byte-input pass's registers)
set -u
export TMPDIR=/tmp
O=gpurun_out/r5e19
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_prove_gpu.py -k "derive or golden or 2_16" > $O/tests.log 2>&1 || { echo "tests failed"; tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 600 tools/prove_opts_ab.sh 4 "PROVE_DERIVE_T2A=1" "PROVE_DERIVE_T2A=2" > $O/prove_ab.txt 2>&1 || { echo "prove ab failed"; tail $O/prove_ab.txt; exit 1; }
cat $O/prove_ab.txt
LIBS="plonk.c_amd/libplonkhip.so plonk.c_amd/build/var/lib_nodrv.so" timeout -k 10 300 tools/c3_lib_ab.sh 3 > $O/c3ab.txt 2>&1 || { echo "c3 ab failed"; cat $O/c3ab.txt; exit 1; }
cat $O/c3ab.txt
echo done
