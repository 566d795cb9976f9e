#!/bin/bash
# round-5 batch 25: the tile-size threshold after the round-5 barrier work -- 2^21 products on
# 2^12 tiles (NTT_T13_MIN_K = 22) against 2^13 (21, the default), prove A/B at 31 calls per median
set -u
export TMPDIR=/tmp
O=gpurun_out/r5e25
mkdir -p $O
PROVE_REPS=31 timeout -k 10 900 tools/prove_opts_ab.sh 4 "NTT_T13_MIN_K=21" "NTT_T13_MIN_K=22" > $O/prove_ab.txt 2>&1 || { echo "prove ab failed"; tail $O/prove_ab.txt; exit 1; }
cat $O/prove_ab.txt
echo done
