#!/bin/bash
# Summarise a tools/profile_bench.sh run (merged back under gpurun_out/prof_<tag>/) into
# the tracked profiles/ directory:  bash tools/collect_profiles.sh <tag> [round] [msms per launch]
set -eu
TAG=$1
R=${2:-$TAG}
P=gpurun_out/prof_$TAG
python3 tools/kstats.py $P/trace/run_results.db --json profiles/${R}_bench_kernel_stats.json > profiles/${R}_bench_kernel_stats.txt
python3 tools/pmc_summary.py $P/pmc/run_results.db msm_dlog_kernel --latest 22 ${3:-40} profiles/msm_pmc_latest.json > profiles/${R}_msm_pmc.json
grep '^{' $P/bench_traced.json > profiles/${R}_bench_traced.json
echo "wrote profiles/${R}_*"
