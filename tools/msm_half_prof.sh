# rocprof A/B of the single-MSM form (PLK_MSM_HALF=0/1) inside the default bench
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out/hp
for h in 0 1 0 1; do
PLK_MSM_HALF=$h timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/hp/t -o run -- python3 bench.py --steps 20 --no-cpu-baseline > /dev/null 2>&1
python3 tools/kstats.py gpurun_out/hp/t/run_results.db | grep "msm_dlog" | sed "s/^/half=$h /"
rm -rf gpurun_out/hp/t
done
