#!/bin/bash
# NTT lab (tuning aid): the C3 shapes (2^20 forward NTT, 8 x 2^20, poly_mul 2^19 x 2^19, 2^22) for the
# library and its tuning variants (tools/build_var.sh), each under a kernel trace so per-kernel
# durations are reported next to the event-timed totals.  Run through gpurun:
#   bash tools/ntt_lab.sh TAG "lib_a lib_b ..." ["ENV=.. ENV2=.."]
set -u
TAG=$1
O=gpurun_out/ntt_lab_$TAG
mkdir -p $O
export TMPDIR=/tmp
for lib in main $2; do
  path=$PWD/plonk.c_amd/libplonkhip.so
  [ "$lib" != main ] && path=$PWD/plonk.c_amd/build/var/$lib.so
  for envs in "${3:-X=0}"; do
    echo "## $lib $envs" >> $O/lab.txt
    env PLK_LIB=$path $envs timeout -k 5 120 python tools/ntt_bench.py --quick >> $O/lab.txt 2>/dev/null || exit 1
    env PLK_LIB=$path $envs timeout -k 5 120 rocprofv3 --kernel-trace -d $O/tr_$lib -o run -- python3 tools/ntt_bench.py --quick > /dev/null 2>&1 || exit 1
    python3 tools/kstats.py $O/tr_$lib/run_results.db wt_ --wide >> $O/lab.txt || exit 1
    rm -rf $O/tr_$lib
  done
done
cat $O/lab.txt
