set -u
mkdir -p gpurun_out/ls
timeout -k 10 400 python -u -m pytest tests/test_polymul_gpu.py tests/test_prove_gpu.py tests/test_ntt_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/ls/tests.log 2>&1; echo "tests rc=$?"; tail -3 gpurun_out/ls/tests.log
for r in 1 2; do
  for v in 1 0; do
    PLK_NTT_LS=$v timeout -k 10 120 python tools/prove_bench.py 20 2>/dev/null | sed "s/^/LS=$v /" || exit 1
  done
done
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/ls/p -o run -- python3 tools/prove_bench.py 20 > /dev/null 2>&1 && python3 tools/prove_breakdown.py gpurun_out/ls/p/run_results.db > gpurun_out/ls/bd1.txt
PLK_NTT_LS=0 timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/ls/q -o run -- python3 tools/prove_bench.py 20 > /dev/null 2>&1 && python3 tools/prove_breakdown.py gpurun_out/ls/q/run_results.db > gpurun_out/ls/bd0.txt
rm -rf gpurun_out/ls/p gpurun_out/ls/q
head -4 gpurun_out/ls/bd1.txt; head -4 gpurun_out/ls/bd0.txt
