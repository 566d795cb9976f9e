#!/bin/bash
# round-5 batch 28: column tables only for two-pass plans -- the 2^12-tile three-pass plans
# (NTT_T13_MIN_K 22 / 28) against references, the 2^20 proof at T13_MIN_K 22, and the NTT /
# poly_mul GPU tests
set -u
export TMPDIR=/tmp
O=gpurun_out/r5e28
mkdir -p $O
timeout -k 10 300 python3 tools/t13_probe.py 22 21 22 > $O/p22.txt 2>&1 || { echo "probe failed"; cat $O/p22.txt; exit 1; }
cat $O/p22.txt
PLK_TUNE="NTT_T13_MIN_K=22" timeout -k 10 120 python3 tools/prove_bench.py 20 > $O/o.json 2>$O/err.txt || { echo "prove failed"; tail $O/err.txt; exit 1; }
python3 -c "import json; d=json.load(open('$O/o.json'))['prove_2^20']; print('[T13=22]', d['median_ms'], d['matches_oracle'])"
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_ntt_gpu.py tests/test_polymul_gpu.py > $O/tests.log 2>&1 || { echo "tests failed"; tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
echo done
