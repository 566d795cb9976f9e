#!/bin/bash
set -u
export TMPDIR=/tmp
O=gpurun_out/r5e3
mkdir -p $O
timeout -k 10 300 tools/c3_lib_ab.sh 3 > $O/c3ab.txt 2>&1 || { echo "c3 ab failed"; cat $O/c3ab.txt; exit 1; }
cat $O/c3ab.txt
timeout -k 10 500 tools/prove_opts_ab.sh 3 "PROVE_EVAL_AGG=0" "PROVE_EVAL_AGG=1" "PROVE_EVAL_AGG=1,PROVE_EARLY_COMMITS=2" > $O/oab.txt 2>&1 || { echo "oab failed"; tail $O/oab.txt; exit 1; }
cat $O/oab.txt
