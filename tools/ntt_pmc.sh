#!/bin/bash
# PMC passes over tools/ntt_bench.py (tuning aid): wave-state and instruction-mix counters
# of the NTT pass kernels.  Each --pmc pass is its own process (no tracing combined).
set -u
O=gpurun_out/ntt_pmc
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES SQ_WAVES -d $O/p1 -o run -- python3 tools/ntt_bench.py > $O/p1.out 2>&1 || exit 1
timeout -k 10 200 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU -d $O/p2 -o run -- python3 tools/ntt_bench.py > $O/p2.out 2>&1 || exit 1
python3 tools/pmc_kernels.py $O/p1/run_results.db wt_ > $O/p1.txt && python3 tools/pmc_kernels.py $O/p2/run_results.db wt_ > $O/p2.txt && rm -rf $O/p1 $O/p2
echo pmc done
