#!/bin/bash
# PMC passes over the prove pipeline at 2^20 gates (tuning aid): per-kernel issue / wait
# counters of the NTT passes and the prover kernels.  Each --pmc pass is its own process.
set -u
O=gpurun_out/prove_pmc
mkdir -p $O
export TMPDIR=/tmp
run() {
  timeout -s KILL 200 rocprofv3 --pmc "$@" -d $O/p -o run -- python3 tools/prove_bench.py 20 > $O/p.out 2>&1 || return 1
  python3 tools/pmc_kernels.py $O/p/run_results.db >> $O/pmc.txt
  rm -rf $O/p
}
: > $O/pmc.txt
run SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES SQ_WAVES || exit 1
run SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INST_CYCLES_VMEM SQ_INSTS_VALU SQ_INSTS_LDS || exit 1
run TCC_HIT_sum TCC_MISS_sum TA_BUSY_avr TA_TA_BUSY_sum || echo "p3 failed"
echo pmc done
