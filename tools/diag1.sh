set -u
mkdir -p gpurun_out/diag1
export TMPDIR=/tmp
timeout -k 10 120 ./tools/bwtest $((16<<20)) > gpurun_out/diag1/bw16.txt 2>&1 || exit 1
timeout -k 10 120 ./tools/bwtest $((128<<20)) > gpurun_out/diag1/bw128.txt 2>&1 || exit 1
timeout -k 10 200 python tools/msm_sweep.py 22 > gpurun_out/diag1/sweep_default.json 2>&1 || exit 1
PLK_MSM_SHARDED=1 timeout -k 10 200 python tools/msm_sweep.py 22 > gpurun_out/diag1/sweep_sharded.json 2>&1 || exit 1
bash tools/profile_bench.sh r01b || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/diag1/prove -o run -- python3 tools/prove_bench.py 20 > gpurun_out/diag1/prove.json 2>&1 || exit 1
echo diag done
