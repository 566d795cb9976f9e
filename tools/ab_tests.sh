#!/bin/bash
# correctness of every variant library first (NTT + poly_mul + prover tests), then A/B timing
set -u
for lib in plonk.c_amd/build/var/lib_*.so; do
  PLK_LIB=$PWD/$lib timeout -k 10 300 python -m pytest tests/test_ntt_gpu.py tests/test_polymul_gpu.py tests/test_prove_gpu.py -q -x > gpurun_out/ab_t.log 2>&1 || { echo "$lib FAILED"; tail -20 gpurun_out/ab_t.log; exit 1; }
  echo "$lib tests ok: $(tail -1 gpurun_out/ab_t.log)"
done
