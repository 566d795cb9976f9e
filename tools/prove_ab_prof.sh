#!/bin/bash
# kernel-span A/B of the prover under rocprofv3 (tuning aid): option NAME at each value given,
# plain and preprocessed (PLK_TUNE="NAME=value": plk_set_option in tools/prove_bench.py)
set -u
export TMPDIR=/tmp
V=${1:-NTT_SHARED_FIX}
mkdir -p gpurun_out/pabp
for r in 1 2; do
for x in ${2:-0 1}; do
  for pre in "" "--pre"; do
    ( export PLK_TUNE="$V=$x"; timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/pabp/p -o run -- python3 tools/prove_bench.py $pre 20 > /dev/null 2>&1 ) || exit 1
    echo "$V=$x pre=${pre:-no}: $(python3 tools/prove_spans.py gpurun_out/pabp/p/run_results.db)"
    rm -rf gpurun_out/pabp/p
  done
done
done
