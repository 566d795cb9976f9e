#!/bin/bash
# A/B timing of the current library against plonk.c_amd/build/var/lib_*.so in ONE box session
# (tuning aid; boxes differ by ~10%, so only same-session comparisons count).
set -u
for rep in 1 2; do
  for lib in plonk.c_amd/libplonkhip.so plonk.c_amd/build/var/lib_*.so; do
    echo "$lib $(PLK_LIB=$PWD/$lib timeout -k 5 120 python tools/${AB_TOOL:-ntt_bench.py} ${AB_ARGS:-} 2>/dev/null)" || exit 1
  done
done
