#!/bin/bash
# round-5 batch 7: round 5's one-launch divisions from round 4's chunk aggregates (PROVE_EVAL_AGG) against the
# two-launch form, alternating; the inverse passes' mod-17 output as arithmetic (build/var/lib_m17a.so)
# against the LDS table, per kernel, three alternations
set -u
export TMPDIR=/tmp
O=gpurun_out/r5e7
mkdir -p $O
timeout -k 10 500 bash tools/prove_opts_ab.sh 4 "PROVE_EVAL_AGG=0" "PROVE_EVAL_AGG=1" > $O/agg.txt 2>&1 || { echo "agg ab failed"; tail $O/agg.txt; exit 1; }
cat $O/agg.txt
for r in 1 2 3; do
  AB_KSUB=wt_inv timeout -k 10 400 bash tools/ab_kernels.sh >> $O/m17.txt 2>&1 || { echo "ab kernels failed"; tail $O/m17.txt; exit 1; }
done
cat $O/m17.txt
echo done
