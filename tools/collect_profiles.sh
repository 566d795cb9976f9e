#!/bin/bash
# Copy the summaries of a tools/round_profile.sh run (gpurun_out/prof_<tag>/) into the tracked
# profiles/ directory:  bash tools/collect_profiles.sh <tag> <round>
set -eu
TAG=$1
R=${2:-$TAG}
P=gpurun_out/prof_$TAG
grep '^{' $P/bench.json > profiles/${R}_bench.json
grep '^{' $P/bench_traced.json > profiles/${R}_bench_traced.json
cp $P/bench_kernel_stats.txt profiles/${R}_bench_kernel_stats.txt
cp $P/bench_kernel_stats.json profiles/${R}_bench_kernel_stats.json
cp $P/msm_pmc.json profiles/${R}_msm_pmc.json
cp $P/msm_pmc_latest.json profiles/msm_pmc_latest.json
cp "$P/prove_2^20_breakdown.txt" "profiles/${R}_prove_2^20_breakdown.txt"
[ -f "$P/prove_2^20_preprocessed_breakdown.txt" ] && cp "$P/prove_2^20_preprocessed_breakdown.txt" "profiles/${R}_prove_2^20_preprocessed_breakdown.txt"
cp $P/ntt_bench.json profiles/${R}_ntt_bench.json
for f in bfly_peak.json prove_ntt_roofline.json prove_ntt_roofline.txt ntt_roofline.json ntt_roofline.txt prove_plan.json; do
  [ -f $P/$f ] && cp $P/$f profiles/${R}_$f
done
tail -1 $P/gpu_tests.log > profiles/${R}_gpu_tests.txt
echo "wrote profiles/${R}_*"
