#!/bin/bash
# prover wall-time A/B on one box (tuning aid): ENV=0 vs ENV=1 (default PLK_NTT_SHARED_FIX),
# plain and preprocessed, alternating; the poly_mul / prover GPU tests first
set -u
export TMPDIR=/tmp
V=${1:-PLK_NTT_SHARED_FIX}
mkdir -p gpurun_out/pab
timeout -k 10 400 python -u -m pytest tests/test_prove_gpu.py tests/test_polymul_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/pab/t.log 2>&1 || { tail -30 gpurun_out/pab/t.log; exit 1; }
tail -1 gpurun_out/pab/t.log
for r in 1 2; do
  for x in 0 1; do
    for pre in "" "--pre"; do
      env $V=$x timeout -k 10 120 python3 tools/prove_bench.py $pre 20 2>/dev/null > gpurun_out/pab/o.json || exit 1
      python3 -c "import json,sys; d=json.load(open('gpurun_out/pab/o.json'))['prove_2^20']; print('$V=$x pre=${pre:-no}', d['ms'], d['median_ms'], d['matches_oracle'])"
    done
  done
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/pab/pp -o run -- python3 tools/prove_bench.py --pre 20 > /dev/null 2>&1 || exit 1
python3 tools/prove_breakdown.py gpurun_out/pab/pp/run_results.db
rm -rf gpurun_out/pab/pp
