#!/bin/bash
# Counter evidence for the prover's NTT kernels at 2^20 gates: four --pmc
# passes over tools/prove_bench.py 20, each its own process (no tracing combined), summarised
# per kernel by tools/ntt_pmc_summary.py against each kernel's algorithmic bytes and butterflies.
#   A: issue / wait split     B: instruction mix + LDS bank conflicts
#   C: FETCH_SIZE (x2 on gfx950 for wide streaming reads)    D: WRITE_SIZE
set -u
O=gpurun_out/ntt_pmc
ARGS=${1:-20}
mkdir -p $O
export TMPDIR=/tmp
run() {
  local tag=$1; shift
  timeout -s KILL 200 rocprofv3 --pmc "$@" -d $O/$tag -o run -- python3 tools/prove_bench.py $ARGS > $O/$tag.out 2>&1 || return 1
}
run A SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAVES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_WAIT_ANY SQ_ACTIVE_INST_ANY || exit 1
run B SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU || exit 1
run C FETCH_SIZE || exit 1
run D WRITE_SIZE || exit 1
# the proof's launch plan (arrays per table pass: grid y counts array groups since round 4)
timeout -k 10 120 python3 tools/prove_plan.py $ARGS > $O/plan.json 2>/dev/null || exit 1
python3 tools/ntt_pmc_summary.py $O/A/run_results.db $O/B/run_results.db $O/C/run_results.db $O/D/run_results.db --plan $O/plan.json > $O/summary.txt || exit 1
rm -rf $O/A $O/B $O/C $O/D
echo "ntt pmc done"
