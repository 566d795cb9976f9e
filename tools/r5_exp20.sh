#!/bin/bash
# round-5 batch 20: host-vs-GPU pacing of a 2^20 proof (HIP runtime trace + kernel trace), both
# A2 B2 modes; then prove A/B with more alternations
set -u
export TMPDIR=/tmp
O=gpurun_out/r5e20
mkdir -p $O
for m in 1 2; do
  PLK_TUNE="PROVE_DERIVE_T2A=$m" timeout -k 10 300 rocprofv3 --kernel-trace --hip-runtime-trace -d $O/t$m -o run -- python3 tools/prove_bench.py 20 > $O/t$m.log 2>&1 || { echo "trace $m failed"; tail $O/t$m.log; exit 1; }
  python3 tools/prove_hostgap.py $O/t$m/run_results.db > $O/hostgap_$m.txt 2>&1 || { echo "hostgap failed"; cat $O/hostgap_$m.txt; exit 1; }
  rm -rf $O/t$m
done
head -40 $O/hostgap_1.txt
timeout -k 10 900 tools/prove_opts_ab.sh 8 "PROVE_DERIVE_T2A=1" "PROVE_DERIVE_T2A=2" > $O/prove_ab.txt 2>&1 || { echo "prove ab failed"; tail $O/prove_ab.txt; exit 1; }
cat $O/prove_ab.txt
echo done
