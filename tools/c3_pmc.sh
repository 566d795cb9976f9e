#!/bin/bash
# Counter passes over config C3 (tools/c3_bench.py: the 2^20 F29 forward transform and poly_mul
# 2^19 x 2^19), each --pmc pass its own process, plus a kernel trace for the durations.
#   A: issue / wait split   B: instruction mix + LDS bank conflicts   C: FETCH_SIZE   D: WRITE_SIZE
set -u
O=gpurun_out/c3_pmc
mkdir -p $O
export TMPDIR=/tmp
run() {
  local tag=$1; shift
  timeout -s KILL 120 rocprofv3 --pmc "$@" -d $O/$tag -o run -- python3 tools/c3_bench.py 20 > $O/$tag.out 2>&1 || return 1
  python3 tools/pmc_kernels.py $O/$tag/run_results.db wt_ > $O/$tag.txt
}
run A SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAVES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_WAIT_ANY SQ_ACTIVE_INST_ANY || exit 1
run B SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU || exit 1
run C FETCH_SIZE || exit 1
run D WRITE_SIZE || exit 1
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/T -o run -- python3 tools/c3_bench.py 20 > $O/T.out 2>&1 || exit 1
python3 tools/kstats.py $O/T/run_results.db wt_ > $O/durations.txt
rm -rf $O/A $O/B $O/C $O/D $O/T
cat $O/durations.txt $O/A.txt $O/B.txt $O/C.txt $O/D.txt
echo "c3 pmc done"
