#!/bin/bash
# round-6 batch 1: the driver's N = 4 / 8 bench runs rehearsed over gloo on one GPU,
# then the default N = 1 bench line as this round's starting point
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r6
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread tests/test_bench_dist_gpu.py \
    > gpurun_out/r6/b1_dist.txt 2>&1 || { tail -50 gpurun_out/r6/b1_dist.txt; exit 1; }
tail -5 gpurun_out/r6/b1_dist.txt
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r6/b1_bench.json 2> gpurun_out/r6/b1_bench.err
