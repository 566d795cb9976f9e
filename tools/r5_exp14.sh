#!/bin/bash
# round-5 batch 14: with the cheaper centre, the shared-operand lo = 0 launch against running those
# passes inside the centre items (NTT_SHARED_FIX=0: one launch fewer), alternating
set -u
export TMPDIR=/tmp
timeout -k 10 600 bash tools/prove_opts_ab.sh 4 "NTT_SHARED_FIX=1" "NTT_SHARED_FIX=0" > gpurun_out/r5e14.txt 2>&1 || { echo "ab failed"; tail gpurun_out/r5e14.txt; exit 1; }
cat gpurun_out/r5e14.txt
