#!/bin/bash
# round-5 experiment batch 1: inverse-pass mod-17 table vs arithmetic (prover A/B), the single
# 2^22 MSM at 16 B per lane (full groups) vs half groups, and the C3 center kernel's counters
set -u
export TMPDIR=/tmp
O=gpurun_out/r5e1
mkdir -p $O
timeout -k 10 400 tools/prove_lib_ab.sh 3 > $O/prove_ab.txt 2>&1 || { echo "prove ab failed"; tail $O/prove_ab.txt; exit 1; }
cat $O/prove_ab.txt
: > $O/single.txt
for cfg in "" "MSM_HALF=0" "MSM_HALF=0,MSM_THREADS=256" "MSM_HALF=0,MSM_MAX_BLOCKS=1024" "MSM_HALF=0,MSM_THREADS=1024" "" "MSM_HALF=0"; do
  PLK_TUNE="$cfg" timeout -k 5 120 python3 tools/msm_single_sweep.py >> $O/single.txt 2>&1 || { echo "failed: $cfg" >> $O/single.txt; exit 1; }
done
cat $O/single.txt
timeout -k 10 600 tools/center_pmc.sh > $O/center_pmc.log 2>&1 || { echo "center pmc failed"; tail $O/center_pmc.log; exit 1; }
echo done
