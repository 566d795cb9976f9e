#!/bin/bash
# round-5 batch 27: where 2^12-tile plans of 2^21+ points go wrong (NTT_T13_MIN_K = 22 / 28)
set -u
export TMPDIR=/tmp
O=gpurun_out/r5e27
mkdir -p $O
timeout -k 10 300 python3 tools/t13_probe.py 22 21 > $O/p22.txt 2>&1; echo "rc $?" >> $O/p22.txt
cat $O/p22.txt
timeout -k 10 300 python3 tools/t13_probe.py 28 21 22 > $O/p28.txt 2>&1; echo "rc $?" >> $O/p28.txt
cat $O/p28.txt
echo done
