# A/B of the swizzled exchange layout (tuning aid): GPU tests of the NTT users, then the prove and
# C3 labs for the library and lib_swz0 (tools/build_var.sh swz0 "-DPLK_NTT_SWZ=0")
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_ntt_gpu.py tests/test_polymul_gpu.py tests/test_prove_gpu.py > gpurun_out/swz_tests.log 2>&1 || { tail -20 gpurun_out/swz_tests.log; exit 1; }
tail -1 gpurun_out/swz_tests.log
bash tools/prove_lab.sh c "lib_swz0" > /dev/null 2>&1
bash tools/prove_lab.sh c2 "lib_swz0" > /dev/null 2>&1
bash tools/ntt_lab.sh s "lib_swz0" > /dev/null 2>&1
cat gpurun_out/prove_lab_c/lab.txt gpurun_out/prove_lab_c2/lab.txt | grep -E "##|span|wt_"
grep -E "##|^\{" gpurun_out/ntt_lab_s/lab.txt
