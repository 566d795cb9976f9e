#!/bin/bash
# C3 A/B between library builds (tuning aid): tools/c3_time.py for libplonkhip.so and every
# build/var/lib_*.so, alternating, ROUNDS rounds
set -u
R=${1:-3}
LIBS=${LIBS:-"plonk.c_amd/libplonkhip.so $(ls plonk.c_amd/build/var/lib_*.so)"}
for r in $(seq $R); do
  for lib in $LIBS; do
    echo "$(basename $lib) $(PLK_LIB=$PWD/$lib timeout -k 5 120 python3 tools/c3_time.py 2>/dev/null | grep '^{')" || exit 1
  done
done
