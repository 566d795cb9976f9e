#!/bin/bash
# PMC passes over tools/ntt_bench.py for the NTT / poly_mul kernels (tuning aid), plus the
# integer-multiply issue-rate probe.  Each --pmc pass is its own process (no tracing combined).
set -u
O=gpurun_out/center_pmc
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 60 ./tools/isa_rate > $O/isa_rate.txt 2>&1 || exit 1
timeout -s KILL 200 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES SQ_WAVES -d $O/p1 -o run -- python3 tools/ntt_bench.py > $O/p1.out 2>&1 || exit 1
timeout -s KILL 200 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU -d $O/p2 -o run -- python3 tools/ntt_bench.py > $O/p2.out 2>&1 || exit 1
timeout -s KILL 200 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_MISC -d $O/p3 -o run -- python3 tools/ntt_bench.py > $O/p3.out 2>&1 || echo "p3 failed"
for p in p1 p2 p3; do [ -f $O/$p/run_results.db ] && python3 tools/pmc_kernels.py $O/$p/run_results.db wt_ > $O/$p.txt; done
rm -rf $O/p1 $O/p2 $O/p3
echo pmc done
