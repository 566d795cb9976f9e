#!/bin/bash
# One GPU call of round-3 work (run through gpurun): each step under its own time limit; a
# failing test lets the next step run, a timeout / abort / crash ends the call.
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
ok() {   # continue only after a clean exit or plain test failures (pytest 1)
  local rc=$1 what=$2
  echo "$what rc=$rc"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $what"; exit $rc; fi
}
for step in "$@"; do
  case $step in
    msm) timeout -k 10 400 python -u -m pytest tests/test_msm_gpu.py -x -v -s --timeout 200 --timeout-method thread > gpurun_out/r3_msm.log 2>&1; ok $? msm
         grep -E "PASS|FAIL|raw fold|Error" gpurun_out/r3_msm.log | tail -30 ;;
    shards) timeout -k 10 300 python -u -m pytest tests/test_shards_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r3_shards.log 2>&1; ok $? shards; tail -3 gpurun_out/r3_shards.log ;;
    gputests) timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r3_gpu_tests.log 2>&1; ok $? gputests; tail -5 gpurun_out/r3_gpu_tests.log ;;
    nttpmc) timeout -k 10 600 ./tools/ntt_pmc_r3.sh 20 > gpurun_out/r3_nttpmc.log 2>&1; ok $? nttpmc; cat gpurun_out/ntt_pmc/summary.txt | head -60 ;;
    bench) timeout -k 10 400 python bench.py > gpurun_out/r3_bench.json 2> gpurun_out/r3_bench.err; ok $? bench ;;
    prove) timeout -k 10 300 python tools/prove_bench.py 20 > gpurun_out/r3_prove.json 2>&1; ok $? prove; cat gpurun_out/r3_prove.json ;;
    proveprof) rm -rf gpurun_out/pp; timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/pp -o run -- python3 tools/prove_bench.py 20 > gpurun_out/r3_pp.json 2>&1; ok $? proveprof
         python3 tools/prove_breakdown.py gpurun_out/pp/run_results.db > gpurun_out/r3_prove_breakdown.txt; cat gpurun_out/r3_prove_breakdown.txt; rm -rf gpurun_out/pp ;;
    nttbench) timeout -k 10 200 python tools/ntt_bench.py > gpurun_out/r3_ntt_bench.json 2>/dev/null; ok $? nttbench; cat gpurun_out/r3_ntt_bench.json | head -c 3000 ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
echo "all steps done"
