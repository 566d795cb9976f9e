#!/bin/bash
# round-5 batch 17: the persistent centre's grid under the new barrier regime (512 resident blocks
# against 768 / 1024 with a dynamic tail), alternating
set -u
export TMPDIR=/tmp
timeout -k 10 700 bash tools/prove_opts_ab.sh 3 "NTT_CENTER_BLOCKS=512" "NTT_CENTER_BLOCKS=768" "NTT_CENTER_BLOCKS=1024" > gpurun_out/r5e17.txt 2>&1 || { echo "ab failed"; tail gpurun_out/r5e17.txt; exit 1; }
cat gpurun_out/r5e17.txt
