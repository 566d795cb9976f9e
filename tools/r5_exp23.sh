#!/bin/bash
# round-5 batch 23: graph replay with the cleared completion word -- prover tests, then prove A/B
# at 31 calls per median (direct / graph / graph + A2 B2 in the t_2 forward pass / that alone)
set -u
export TMPDIR=/tmp
O=gpurun_out/r5e23
mkdir -p $O
timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_prove_gpu.py -k "graph or derive or golden" > $O/tests.log 2>&1 || { echo "tests failed"; tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
PROVE_REPS=31 timeout -k 10 1000 tools/prove_opts_ab.sh 6 "PROVE_GRAPH=0" "PROVE_GRAPH=1" "PROVE_GRAPH=1,PROVE_DERIVE_T2A=2" "PROVE_DERIVE_T2A=2" > $O/prove_ab.txt 2>&1 || { echo "prove ab failed"; tail $O/prove_ab.txt; exit 1; }
cat $O/prove_ab.txt
echo done
