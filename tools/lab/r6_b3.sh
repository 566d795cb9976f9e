#!/bin/bash
# round-6 batch 3: (1) the two-pass data-movement floor at more tiles per CU (tools/floor_lab.hip,
# VERDICT r5 #3); (2) the drop-in GPU tests left out of batch 2; (3) the last inverse passes' column
# factors derived instead of read (build/var/lib_coli.so): parity, alternating prove
# medians, kernel breakdown and FETCH / WRITE counters against the default build; (4) the default
# build's four PMC passes over the prover with the centre's butterflies and bytes
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r6
mkdir -p $O
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 120 ./tools/floor_lab > $O/b3_floor.txt 2>&1 || { cat $O/b3_floor.txt; exit 1; }
cat $O/b3_floor.txt
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu \
    tests/test_dropin_gpu.py tests/test_reference_suite.py > $O/b3_dropin.txt 2>&1 || { tail -40 $O/b3_dropin.txt; exit 1; }
tail -2 $O/b3_dropin.txt
PLK_LIB=$PWD/plonk.c_amd/build/var/lib_coli.so timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
    tests/test_polymul_gpu.py tests/test_prove_gpu.py > $O/b3_coli_tests.txt 2>&1 || { tail -40 $O/b3_coli_tests.txt; exit 1; }
tail -2 $O/b3_coli_tests.txt
LIBS="plonk.c_amd/libplonkhip.so plonk.c_amd/build/var/lib_coli.so" PB_ARGS=20 timeout -k 10 900 bash tools/prove_lib_ab.sh 3 > $O/b3_coli_ab.txt 2>&1 || { tail -30 $O/b3_coli_ab.txt; exit 1; }
cat $O/b3_coli_ab.txt
for lib in plonk.c_amd/libplonkhip.so plonk.c_amd/build/var/lib_coli.so; do
  t=$(basename $lib .so)
  for c in FETCH_SIZE WRITE_SIZE; do
    PLK_LIB=$PWD/$lib timeout -s KILL 200 rocprofv3 --pmc $c -d $O/pmc_${t}_$c -o run -- python3 tools/prove_bench.py 20 > $O/pmc_${t}_$c.out 2>&1 || { echo "pmc $t $c failed"; tail $O/pmc_${t}_$c.out; exit 1; }
    python3 - "$O/pmc_${t}_$c/run_results.db" "$t" "$c" <<'PY'
import sqlite3, sys
from collections import defaultdict
db, t, c = sys.argv[1:4]
con = sqlite3.connect(db)
acc = defaultdict(list)
for name, v in con.execute("select name, counter_value from pmc_events where counter_name = ?", (c,)):
    if "wt_inv_kernel" in name:
        acc[name.split("(")[0]].append(float(v))
for k, v in sorted(acc.items()):
    print("%-10s %-10s %-70s mean %.4g KiB over %d launches" % (t, c, k[:70], sum(v) / len(v), len(v)))
PY
    rm -rf $O/pmc_${t}_$c
  done
done
timeout -k 10 900 bash tools/ntt_pmc_r4.sh 20 > $O/b3_pmc.txt 2>&1 || { tail -20 $O/b3_pmc.txt; exit 1; }
cp gpurun_out/ntt_pmc/summary.txt $O/b3_ntt_pmc_summary.txt
cat $O/b3_ntt_pmc_summary.txt | cut -c1-160
