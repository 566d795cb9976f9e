#!/bin/bash
# round-5 batch 5: the two-half C3 center (build/var/lib_dual.so) against the round-4 form -- its
# poly_mul / NTT tests, then C3 timings alternating --, the inverse passes' mod-17 byte output as
# LDS table vs 24-bit arithmetic (build/var/lib_m17a.so, prover A/B), the single 2^22 MSM at 16 B
# per lane (MSM_HALF=0, several geometries) vs half groups, and C3's counter passes
set -u
export TMPDIR=/tmp
O=gpurun_out/r5e5
mkdir -p $O
PLK_LIB=$PWD/plonk.c_amd/build/var/lib_dual.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_polymul_gpu.py tests/test_ntt_gpu.py > $O/dual_tests.log 2>&1 || { echo "dual tests failed"; tail -30 $O/dual_tests.log; exit 1; }
tail -1 $O/dual_tests.log
PLK_LIB=$PWD/plonk.c_amd/build/var/lib_lor3.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_ntt_gpu.py > $O/lor3_tests.log 2>&1 || { echo "lor3 tests failed"; tail -30 $O/lor3_tests.log; exit 1; }
tail -1 $O/lor3_tests.log
timeout -k 10 300 tools/c3_lib_ab.sh 3 > $O/c3ab.txt 2>&1 || { echo "c3 ab failed"; cat $O/c3ab.txt; exit 1; }
cat $O/c3ab.txt
LIBS="plonk.c_amd/libplonkhip.so plonk.c_amd/build/var/lib_m17a.so" timeout -k 10 400 tools/prove_lib_ab.sh 3 > $O/prove_ab.txt 2>&1 || { echo "prove ab failed"; tail $O/prove_ab.txt; exit 1; }
cat $O/prove_ab.txt
: > $O/single.txt
for cfg in "" "MSM_HALF=0" "MSM_HALF=0,MSM_THREADS=256" "MSM_HALF=0,MSM_THREADS=1024" "MSM_HALF=0,MSM_GROUPS=2" "" "MSM_HALF=0"; do
  PLK_TUNE="$cfg" timeout -k 5 120 python3 tools/msm_single_sweep.py >> $O/single.txt 2>&1 || { echo "failed: $cfg" >> $O/single.txt; cat $O/single.txt; exit 1; }
done
cat $O/single.txt
timeout -k 10 300 tools/c3_pmc.sh > $O/c3.log 2>&1 || { echo "c3 pmc failed"; tail $O/c3.log; exit 1; }
cp -r gpurun_out/c3_pmc $O/c3_pmc_r4form
PLK_LIB=$PWD/plonk.c_amd/build/var/lib_dual.so timeout -k 10 300 tools/c3_pmc.sh > $O/c3_dual.log 2>&1 || { echo "c3 dual pmc failed"; tail $O/c3_dual.log; exit 1; }
cat $O/c3.log $O/c3_dual.log
echo done
