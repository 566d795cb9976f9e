#!/bin/bash
# MSM launch-shape sweep on the GPU box (tuning aid): correctness first, then
# tools/msm_sweep.py under several PLK_MSM_* settings.  Output: gpurun_out/tune_<tag>/
set -u
TAG=${1:-t}
O=gpurun_out/tune_$TAG
mkdir -p $O
timeout -k 10 300 python -m pytest tests/test_msm_gpu.py tests/test_prove_gpu.py tests/test_dropin_gpu.py -q -x > $O/tests.log 2>&1 || { echo "tests failed"; tail -30 $O/tests.log; exit 1; }
run() {
  local name=$1; shift
  env "$@" timeout -k 10 200 python tools/msm_sweep.py 22 > $O/$name.json 2> $O/$name.err || { echo "sweep $name failed"; exit 1; }
  echo "$name $(cat $O/$name.json)"
}
run default PLK_MSM_X=0
run g1 PLK_MSM_G=1
run g2 PLK_MSM_G=2
run t512b512 PLK_MSM_THREADS=512 PLK_MSM_MAX_BLOCKS=512
run t512b512g2 PLK_MSM_THREADS=512 PLK_MSM_MAX_BLOCKS=512 PLK_MSM_G=2
run t1024b512 PLK_MSM_MAX_BLOCKS=512
run t256b1024 PLK_MSM_THREADS=256 PLK_MSM_MAX_BLOCKS=1024
echo tune done
