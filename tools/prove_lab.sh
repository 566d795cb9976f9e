#!/bin/bash
# Prover lab (tuning aid): the 2^20 prove breakdown (rocprofv3 kernel trace of tools/prove_bench.py)
# for the library and its tuning variants (tools/build_var.sh).  Run through gpurun:
#   bash tools/prove_lab.sh TAG "lib_a lib_b ..."
set -u
TAG=$1
O=gpurun_out/prove_lab_$TAG
mkdir -p $O
export TMPDIR=/tmp
: > $O/lab.txt
for lib in main $2; do
  path=$PWD/plonk.c_amd/libplonkhip.so
  [ "$lib" != main ] && path=$PWD/plonk.c_amd/build/var/$lib.so
  echo "## $lib" >> $O/lab.txt
  env PLK_LIB=$path timeout -k 5 200 rocprofv3 --kernel-trace -d $O/tr_$lib -o run -- python3 tools/prove_bench.py 20 > $O/out_$lib.json 2>&1 || { echo "failed $lib" >> $O/lab.txt; tail -5 $O/out_$lib.json >> $O/lab.txt; continue; }
  python3 tools/prove_breakdown.py $O/tr_$lib/run_results.db >> $O/lab.txt || exit 1
  rm -rf $O/tr_$lib
done
cat $O/lab.txt
