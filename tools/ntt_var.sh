#!/bin/bash
# NTT variant sweep (tuning aid): ntt_bench for library variants x radix bits.
set -u
for lib in plonk.c_amd/libplonkhip.so plonk.c_amd/build/var/lib_*.so; do
  for r in ${RADIX:-2 3 4}; do
    echo "$lib R=$r $(PLK_LIB=$PWD/$lib PLK_NTT_RADIX_BITS=$r timeout -k 5 120 python tools/ntt_bench.py 2>/dev/null)" || exit 1
  done
done
