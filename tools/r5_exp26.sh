#!/bin/bash
# round-5 batch 26: the 2^20 proof with 2^21 products on 2^12 tiles (NTT_T13_MIN_K = 22, three-pass
# plans) -- which setting gives a wrong proof: the A2 B2 mode, and the round-start library
set -u
export TMPDIR=/tmp
O=gpurun_out/r5e26
mkdir -p $O
for cfg in "NTT_T13_MIN_K=22,PROVE_DERIVE_T2A=1" "NTT_T13_MIN_K=22,PROVE_DERIVE_T2A=2" "NTT_T13_MIN_K=22,PROVE_DERIVE_T2A=0" "NTT_T13_MIN_K=21"; do
  PLK_TUNE="$cfg" timeout -k 10 120 python3 tools/prove_bench.py 20 > $O/o.json 2>$O/err.txt || { echo "failed $cfg"; tail $O/err.txt; exit 1; }
  python3 -c "import json; d=json.load(open('$O/o.json'))['prove_2^20']; print('[$cfg]', d['median_ms'], d['matches_oracle'])"
done
if [ -f plonk.c_amd/build/old/libplonkhip.so ]; then
  PLK_LIB=$PWD/plonk.c_amd/build/old/libplonkhip.so PLK_TUNE="NTT_T13_MIN_K=22" timeout -k 10 120 python3 tools/prove_bench.py 20 > $O/o.json 2>$O/err.txt || { echo "failed old"; tail $O/err.txt; exit 1; }
  python3 -c "import json; d=json.load(open('$O/o.json'))['prove_2^20']; print('[old lib, T13=22]', d['median_ms'], d['matches_oracle'])"
fi
echo done
