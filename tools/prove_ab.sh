#!/bin/bash
# prover wall-time A/B on one box (tuning aid): completion-word polling vs stream synchronize,
# plain and preprocessed, alternating
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/pab
timeout -k 10 300 python -u -m pytest tests/test_prove_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/pab/t.log 2>&1 || { tail -30 gpurun_out/pab/t.log; exit 1; }
tail -1 gpurun_out/pab/t.log
for r in 1 2; do
  for sync in 0 1; do
    for pre in "" "--pre"; do
      PLK_PROVE_SYNC=$sync timeout -k 10 120 python3 tools/prove_bench.py $pre 20 2>/dev/null > gpurun_out/pab/o.json || exit 1
      python3 -c "import json,sys; d=json.load(open('gpurun_out/pab/o.json'))['prove_2^20']; print('sync=$sync pre=${pre:-no}', d['ms'], d['median_ms'], d['matches_oracle'])"
    done
  done
done
