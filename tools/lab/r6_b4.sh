#!/bin/bash
# round-6 batch 4: (1) the derived inverse column factors (build/var/lib_coli.so) against the table,
# per kernel over every launch of two alternating kernel traces each; (2) counters of the floor lab's
# configurations (1, 2 and 4 tiles per CU); (3) config C3's counter passes (tools/c3_pmc.sh)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r6
mkdir -p $O
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
for r in 1 2; do
  for lib in plonk.c_amd/libplonkhip.so plonk.c_amd/build/var/lib_coli.so; do
    PLK_LIB=$PWD/$lib timeout -k 10 200 rocprofv3 --kernel-trace -d $O/abk -o run -- python3 tools/prove_bench.py 20 > $O/abk.out 2>&1 \
      || { echo "$lib failed"; tail $O/abk.out; exit 1; }
    echo "== round $r $(basename $lib) $(grep -o '"median_ms": [0-9.]*' $O/abk.out | head -1)"
    python3 tools/kstats.py $O/abk/run_results.db wt_ | cut -c1-150
    rm -rf $O/abk
  done
done > $O/b4_coli_kernels.txt
cat $O/b4_coli_kernels.txt
for pass in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAVES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY" "FETCH_SIZE" "WRITE_SIZE"; do
  tag=$(echo $pass | cut -d' ' -f1)
  timeout -s KILL 120 rocprofv3 --pmc $pass -d $O/fl_$tag -o run -- ./tools/floor_lab 6 > $O/fl_$tag.out 2>&1 || { echo "floor pmc $tag failed"; tail $O/fl_$tag.out; exit 1; }
  python3 tools/pmc_kernels.py $O/fl_$tag/run_results.db k_ > $O/b4_floor_pmc_$tag.txt
  rm -rf $O/fl_$tag
done
cat $O/b4_floor_pmc_*.txt | cut -c1-260
timeout -k 10 600 bash tools/c3_pmc.sh > $O/b4_c3_pmc.txt 2>&1 || { tail -20 $O/b4_c3_pmc.txt; exit 1; }
cat $O/b4_c3_pmc.txt | cut -c1-250
