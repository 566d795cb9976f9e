#!/bin/bash
# round-6 batch 10: the shared-operand launch filling its last round of blocks (build/var/lib_fill.so,
# PLK_NTT_FIX_FILL=1) against the default: parity, alternating prove medians, kernel breakdowns
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r6
mkdir -p $O
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
PLK_LIB=$PWD/plonk.c_amd/build/var/lib_fill.so timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
    tests/test_prove_gpu.py tests/test_polymul_gpu.py -k "2_20 or batch or shape or preprocessed or random" > $O/b10_tests.txt 2>&1 \
    || { tail -30 $O/b10_tests.txt; exit 1; }
tail -2 $O/b10_tests.txt
LIBS="plonk.c_amd/libplonkhip.so plonk.c_amd/build/var/lib_fill.so" PB_ARGS=20 timeout -k 10 900 bash tools/prove_lib_ab.sh 4 > $O/b10_ab.txt 2>&1 \
    || { tail -30 $O/b10_ab.txt; exit 1; }
cat $O/b10_ab.txt
