#!/bin/bash
# End-of-milestone GPU pass (run through gpurun): GPU tests, the default bench, its rocprofv3
# kernel trace + a separate FETCH_SIZE PMC pass, and the 2^20 prove breakdown.  Summaries are
# written on the box (the raw databases are deleted there: gpurun_out/ must stay < 64 MiB);
# copy them into profiles/ with tools/collect_profiles.sh <tag> <round>.
set -u
TAG=${1:-r01}
O=gpurun_out/prof_$TAG
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 500 python -m pytest tests -m gpu -q > $O/gpu_tests.log 2>&1 || { echo "gpu tests failed"; tail -30 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
# the PMC pass first: bench.py reads roofline.traffic from profiles/msm_pmc_latest.json only when
# it was measured for the current kernel source, so the bench lines below carry it
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE -d $O/pmc -o run -- python3 bench.py --profile-only > $O/pmc.out 2>&1 || exit 1
python3 tools/pmc_summary.py $O/pmc/run_results.db msm_dlog_kernel --latest 22 160 $O/msm_pmc_latest.json > $O/msm_pmc.json || exit 1
cp $O/msm_pmc_latest.json profiles/msm_pmc_latest.json
timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail $O/bench.err; exit 1; }
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/trace -o run -- python3 bench.py > $O/bench_traced.json 2> $O/bench_traced.err || exit 1
python3 tools/kstats.py $O/trace/run_results.db --json $O/bench_kernel_stats.json > $O/bench_kernel_stats.txt || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prove -o run -- python3 tools/prove_bench.py 20 > $O/prove.json 2>&1 || exit 1
python3 tools/prove_breakdown.py $O/prove/run_results.db > $O/prove_2^20_breakdown.txt || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prove_pre -o run -- python3 tools/prove_bench.py --pre 20 > $O/prove_pre.json 2>&1 || exit 1
python3 tools/prove_breakdown.py $O/prove_pre/run_results.db > $O/prove_2^20_preprocessed_breakdown.txt || exit 1
timeout -k 10 60 ./tools/bfly_peak > $O/bfly_peak.json || exit 1
timeout -k 10 120 python3 tools/prove_plan.py 20 > $O/prove_plan.json 2>/dev/null || exit 1
python3 tools/ntt_roofline.py $O/prove/run_results.db $O/bfly_peak.json --prove --plan $O/prove_plan.json --json $O/prove_ntt_roofline.json > $O/prove_ntt_roofline.txt || exit 1
timeout -k 10 200 python tools/ntt_bench.py > $O/ntt_bench.json 2>/dev/null || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/ntt -o run -- python3 tools/ntt_bench.py --plan $O/ntt_plan.json > /dev/null 2>&1 || exit 1
python3 tools/ntt_roofline.py $O/ntt/run_results.db $O/bfly_peak.json --plan $O/ntt_plan.json --json $O/ntt_roofline.json > $O/ntt_roofline.txt || exit 1
rm -rf $O/trace $O/pmc $O/prove $O/prove_pre $O/ntt
echo "round profile $TAG done"
