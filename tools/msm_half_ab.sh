set -e
export TMPDIR=/tmp
mkdir -p gpurun_out/ab
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_msm_gpu.py tests/test_dropin_gpu.py tests/test_prove_gpu.py > gpurun_out/ab/tests.log 2>&1 || { tail -30 gpurun_out/ab/tests.log; exit 1; }
tail -1 gpurun_out/ab/tests.log
for r in 1 2; do
for h in 0 1; do
PLK_MSM_HALF=$h timeout -k 10 200 python bench.py --steps 20 --no-cpu-baseline > gpurun_out/ab/b_$h_$r.json 2>/dev/null
python3 -c "
import json,sys; d=json.loads([l for l in open('gpurun_out/ab/b_$h_$r.json') if l.startswith('{')][0]); c=d['components']
print('half=$h', d['value'], c['msm_2^22_one_per_launch']['device_us_per_msm'], c['msm_2^16']['device_us_per_msm'], c['prove_2^20_gates']['ms'])"
done; done
