#!/bin/bash
# Run the MSM lab binaries (built in the container) under several launch shapes.
set -u
O=gpurun_out/lab_${1:-a}
mkdir -p $O
for cfg in ${CFGS:-"PLK_MSM_X=0" "PLK_MSM_G=1" "PLK_MSM_THREADS=1024 PLK_MSM_MAX_BLOCKS=256" "PLK_MSM_THREADS=256 PLK_MSM_G=4"}; do
  echo "## $cfg"
  for d in ${DIAGS:-0 1 2 3}; do
    env $cfg timeout -k 5 60 ./tools/msm_lab_d$d 22 || exit 1
  done
done > $O/lab.txt 2>&1
cat $O/lab.txt
