#!/bin/bash
# round-6 batch 13: the centre loading the next item's A during this item's inverse pass
# (build/var/lib_cpf.so, PLK_NTT_CENTER_PF=1, 4-5 VGPRs spilled) against the default
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r6
mkdir -p $O
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
PLK_LIB=$PWD/plonk.c_amd/build/var/lib_cpf.so timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
    tests/test_prove_gpu.py -k "2_20 or shape or preprocessed" > $O/b13_tests.txt 2>&1 || { tail -30 $O/b13_tests.txt; exit 1; }
tail -1 $O/b13_tests.txt
LIBS="plonk.c_amd/libplonkhip.so plonk.c_amd/build/var/lib_cpf.so" PB_ARGS=20 timeout -k 10 900 bash tools/prove_lib_ab.sh 4 > $O/b13_ab.txt 2>&1 \
    || { tail -30 $O/b13_ab.txt; exit 1; }
cat $O/b13_ab.txt
