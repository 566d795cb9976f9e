#!/bin/bash
# Tuning round trip (run through gpurun): parity of the NTT / poly_mul / prover tests on the
# current library, then same-session A/B timing against plonk.c_amd/build/var/lib_*.so.
set -u
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_ntt_gpu.py tests/test_polymul_gpu.py tests/test_prove_gpu.py -q -x --timeout 120 --timeout-method thread > gpurun_out/ab_t.log 2>&1 || { echo "tests FAILED"; tail -30 gpurun_out/ab_t.log; exit 1; }
echo "tests ok: $(tail -1 gpurun_out/ab_t.log)"
AB_TOOL=prove_bench.py AB_ARGS=20 bash tools/ab.sh || exit 1
AB_TOOL=ntt_bench.py AB_ARGS= bash tools/ab.sh || exit 1
