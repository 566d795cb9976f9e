#!/bin/bash
# Profile bench.py on the GPU box (run through gpurun).  Raw rocprofv3 output goes under
# gpurun_out/prof_<tag>/ (merged back by gpurun); summarise locally with
#   python tools/kstats.py gpurun_out/prof_<tag>/trace/run_results.db > profiles/...
# Kernel trace + stats of the default bench command, then a SEPARATE PMC pass (FETCH_SIZE,
# never combined with tracing) of the timed MSM loop only.
set -u
TAG=${1:-r01}
OUT=gpurun_out/prof_$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run -- python3 bench.py \
  > "$OUT/bench_traced.json" 2> "$OUT/bench_traced.err" || exit 1
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE -d "$OUT/pmc" -o run -- python3 bench.py --profile-only \
  > "$OUT/pmc.out" 2>&1 || exit 1
echo "profile $TAG done"
