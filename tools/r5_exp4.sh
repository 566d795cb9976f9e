#!/bin/bash
# full GPU suite, then the round-5 A/Bs (agg-divide modes; C3 center against the round-4 form)
set -u
export TMPDIR=/tmp
O=gpurun_out/r5e4
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu tests > $O/tests.log 2>&1 || { echo "tests failed"; tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 200 tools/c3_lib_ab.sh 2 > $O/c3ab.txt 2>&1 || { echo "c3 ab failed"; cat $O/c3ab.txt; exit 1; }
cat $O/c3ab.txt
timeout -k 10 500 tools/prove_opts_ab.sh 3 "PROVE_EVAL_AGG=0" "PROVE_EVAL_AGG=1" "PROVE_EVAL_AGG=1,PROVE_EARLY_COMMITS=2" > $O/oab.txt 2>&1 || { echo "oab failed"; tail $O/oab.txt; exit 1; }
cat $O/oab.txt
