#!/bin/bash
# round-5 batch 22: the proof as a captured HIP graph (PROVE_GRAPH = 1) -- the prover tests, prove
# A/B (direct launches / graph / graph + A2 B2 in the t_2 forward pass), and the graph's kernel
# timeline (kernel + HIP runtime trace)
set -u
export TMPDIR=/tmp
O=gpurun_out/r5e22
mkdir -p $O
timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_prove_gpu.py > $O/tests.log 2>&1 || { echo "tests failed"; tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 900 tools/prove_opts_ab.sh 6 "PROVE_GRAPH=0" "PROVE_GRAPH=1" "PROVE_GRAPH=1,PROVE_DERIVE_T2A=2" > $O/prove_ab.txt 2>&1 || { echo "prove ab failed"; tail $O/prove_ab.txt; exit 1; }
cat $O/prove_ab.txt
PLK_TUNE="PROVE_GRAPH=1" timeout -k 10 300 rocprofv3 --kernel-trace --hip-runtime-trace -d $O/tg -o run -- python3 tools/prove_bench.py 20 > $O/tg.log 2>&1 || { echo "trace failed"; tail $O/tg.log; exit 1; }
python3 tools/prove_hostgap.py $O/tg/run_results.db > $O/hostgap_graph.txt 2>&1 || { echo "hostgap failed"; cat $O/hostgap_graph.txt; exit 1; }
rm -rf $O/tg
head -60 $O/hostgap_graph.txt
echo done
