#!/bin/bash
# Prover round trip (run through gpurun): prover + drop-in parity, timing, ordered kernel timeline.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_prove_gpu.py tests/test_dropin_gpu.py -q -x --timeout 120 --timeout-method thread > gpurun_out/pc_t.log 2>&1 || { echo "tests FAILED"; tail -30 gpurun_out/pc_t.log; exit 1; }
echo "tests ok: $(tail -1 gpurun_out/pc_t.log)"
timeout -k 10 120 python tools/prove_bench.py 20 | cut -c1-80 || exit 1
timeout -k 10 200 rocprofv3 --kernel-trace -d gpurun_out/tl -o run -- python3 tools/prove_bench.py 20 > gpurun_out/tl.out 2>&1 || exit 1
python3 tools/prove_timeline.py gpurun_out/tl/run_results.db > gpurun_out/prove_timeline.txt; rm -rf gpurun_out/tl
