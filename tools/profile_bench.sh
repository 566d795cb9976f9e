#!/bin/bash
# Profile bench.py on the GPU box (run via gpurun).  Writes raw rocprofv3 output under
# gpurun_out/<tag>/ and summaries under profiles/ (copy back and commit those).
#   kernel trace + stats of the default bench command, and a separate PMC pass (FETCH_SIZE,
#   never combined with tracing) of the timed MSM loop only.
set -u
TAG=${1:-r01}
OUT=gpurun_out/prof_$TAG
mkdir -p "$OUT" profiles
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run -- python3 bench.py > "$OUT/bench_traced.json" 2> "$OUT/bench_traced.err" || exit 1
python3 tools/kstats.py "$OUT"/trace/run_results.db --json "profiles/kernel_stats_$TAG.json" > "profiles/kernel_stats_$TAG.txt" || exit 1
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE -d "$OUT/pmc" -o run -- python3 bench.py --profile-only > "$OUT/pmc.out" 2>&1 || exit 1
python3 tools/pmc_summary.py "$OUT"/pmc/run_results.db > "profiles/pmc_fetch_$TAG.json" || exit 1
echo "profile $TAG done"
