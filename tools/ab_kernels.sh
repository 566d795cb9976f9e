#!/bin/bash
# Per-kernel A/B (tuning aid): rocprofv3 kernel trace of ${AB_TOOL:-prove_bench.py} for each
# library, summarised on the box for kernels matching ${AB_KSUB:-wt_}.
set -u
export TMPDIR=/tmp
for lib in plonk.c_amd/libplonkhip.so plonk.c_amd/build/var/lib_*.so; do
  PLK_LIB=$PWD/$lib timeout -k 10 200 rocprofv3 --kernel-trace -d gpurun_out/abk -o run -- python3 tools/${AB_TOOL:-prove_bench.py} ${AB_ARGS:-20} > gpurun_out/abk.out 2>&1 || { echo "$lib failed"; tail gpurun_out/abk.out; exit 1; }
  echo "== $lib $(grep '^{' gpurun_out/abk.out | head -c 120)"
  python3 tools/kstats.py gpurun_out/abk/run_results.db ${AB_KSUB:-wt_} | awk '{print "   " $0}' | cut -c1-150
  rm -rf gpurun_out/abk
done
