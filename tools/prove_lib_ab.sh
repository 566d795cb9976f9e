#!/bin/bash
# Prover wall-time A/B on one box between library builds (tuning aid):
#   tools/prove_lib_ab.sh [rounds]    -- plonk.c_amd/libplonkhip.so against every build/var/lib_*.so
# alternating plain 2^20 proofs (median of 9 calls each, the bench's prove_component), then a rocprof
# kernel breakdown of each build.
set -u
export TMPDIR=/tmp
R=${1:-3}
O=gpurun_out/lab
mkdir -p $O
LIBS=${LIBS:-"plonk.c_amd/libplonkhip.so $(ls plonk.c_amd/build/var/lib_*.so)"}
for r in $(seq $R); do
  for lib in $LIBS; do
    PLK_LIB=$PWD/$lib timeout -k 10 120 python3 tools/prove_bench.py ${PB_ARGS:-20} 2>/dev/null > $O/o.json || { echo "$lib failed"; exit 1; }
    python3 -c "import json; d=json.load(open('$O/o.json')); k=sorted(d)[-1]; d=d[k]; print('$(basename $lib)', k, d['median_ms'], d['best_ms'], d['matches_oracle'])"
  done
done
for lib in $LIBS; do
  PLK_LIB=$PWD/$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/pp -o run -- python3 tools/prove_bench.py 20 > /dev/null 2>&1 || exit 1
  echo "== $lib"
  python3 tools/prove_breakdown.py $O/pp/run_results.db
  rm -rf $O/pp
done
