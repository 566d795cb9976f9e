#!/bin/bash
# Prover wall-time A/B on one box between two PLK_TUNE settings (plk_set_option, tuning aid):
#   tools/prove_tune_ab.sh "A_SETTING" "B_SETTING" [rounds]   e.g. "PROVE_DERIVE_T2A=0" "PROVE_DERIVE_T2A=1"
# alternating plain / preprocessed 2^20 proofs (median of 9 calls each), then a rocprof kernel
# breakdown of each setting.
set -u
export TMPDIR=/tmp
A=$1; B=$2; R=${3:-3}
O=gpurun_out/tab
mkdir -p $O
for r in $(seq $R); do
  for x in "$A" "$B"; do
    for pre in "" "--pre"; do
      PLK_TUNE="$x" timeout -k 10 120 python3 tools/prove_bench.py $pre 20 2>/dev/null > $O/o.json || exit 1
      python3 -c "import json; d=json.load(open('$O/o.json'))['prove_2^20']; print('$x pre=${pre:-no}', d['median_ms'], d['best_ms'], d['matches_oracle'])"
    done
  done
done
for x in "$A" "$B"; do
  PLK_TUNE="$x" timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/pp -o run -- python3 tools/prove_bench.py 20 > /dev/null 2>&1 || exit 1
  echo "== $x"
  python3 tools/prove_breakdown.py $O/pp/run_results.db
  rm -rf $O/pp
done
