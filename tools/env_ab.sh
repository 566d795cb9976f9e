#!/bin/bash
# Same-session A/B over environment settings (tuning aid):
#   AB_TOOL=prove_bench.py AB_ARGS=20 bash tools/env_ab.sh "" "PLK_X=1" "PLK_X=2"
set -u
for rep in 1 2; do
  for spec in "$@"; do
    echo "[$spec] $(env $spec timeout -k 5 120 python tools/${AB_TOOL:-ntt_bench.py} ${AB_ARGS:-} 2>/dev/null | cut -c1-${AB_CUT:-400})" || exit 1
  done
done
