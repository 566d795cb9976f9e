#!/bin/bash
# Prover wall-time A/B on one box between several PLK_TUNE settings (tuning aid):
#   tools/prove_opts_ab.sh ROUNDS "A_SETTING" "B_SETTING" ...
# alternating plain 2^20 proofs (median of 9 calls each), then a rocprof breakdown of each setting
set -u
export TMPDIR=/tmp
R=$1; shift
O=gpurun_out/oab
mkdir -p $O
for r in $(seq $R); do
  for x in "$@"; do
    PLK_TUNE="$x" timeout -k 10 120 python3 tools/prove_bench.py 20 2>/dev/null > $O/o.json || exit 1
    python3 -c "import json; d=json.load(open('$O/o.json'))['prove_2^20']; print('[$x]', d['median_ms'], d['best_ms'], d['matches_oracle'])"
  done
done
for x in "$@"; do
  PLK_TUNE="$x" timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/pp -o run -- python3 tools/prove_bench.py 20 > /dev/null 2>&1 || exit 1
  echo "== [$x]"
  python3 tools/prove_breakdown.py $O/pp/run_results.db
  rm -rf $O/pp
done
