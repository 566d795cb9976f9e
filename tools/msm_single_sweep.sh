#!/bin/bash
# Launch-geometry sweep of the single 2^22-point MSM (tools/msm_single_sweep.py per setting).
set -u
O=gpurun_out/msm_sweep1
mkdir -p $O
: > $O/sweep.txt
for cfg in "" "PLK_MSM_HALF=0" "PLK_MSM_THREADS=256" "PLK_MSM_THREADS=1024" "PLK_MSM_COPIES=8" \
           "PLK_MSM_MAX_BLOCKS=256" "PLK_MSM_MAX_BLOCKS=1024" "PLK_MSM_HALF=0 PLK_MSM_THREADS=1024" \
           "PLK_MSM_THREADS=256 PLK_MSM_MAX_BLOCKS=1024" ""; do
  env $cfg timeout -k 5 120 python3 tools/msm_single_sweep.py >> $O/sweep.txt 2>/dev/null || { echo "failed: $cfg" >> $O/sweep.txt; }
done
cat $O/sweep.txt
