#!/bin/bash
# round-5 batch 21: host-vs-GPU pacing of a 2^20 proof (HIP runtime trace + kernel trace)
set -u
export TMPDIR=/tmp
O=gpurun_out/r5e21
mkdir -p $O
for m in 1; do
  PLK_TUNE="PROVE_DERIVE_T2A=$m" timeout -k 10 300 rocprofv3 --kernel-trace --hip-runtime-trace -d $O/t$m -o run -- python3 tools/prove_bench.py 20 > $O/t$m.log 2>&1 || { echo "trace $m failed"; tail $O/t$m.log; exit 1; }
  python3 tools/prove_hostgap.py $O/t$m/run_results.db > $O/hostgap_$m.txt 2>&1 || { echo "hostgap failed"; cat $O/hostgap_$m.txt; exit 1; }
  rm -rf $O/t$m
done
cat $O/hostgap_1.txt
echo done
