# host-buffer API check (tuning aid): drop-in / polyops / MSM / poly_mul GPU tests, then the bench host-call numbers
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_dropin_gpu.py tests/test_polyops_gpu.py tests/test_msm_gpu.py tests/test_polymul_gpu.py > gpurun_out/hc_tests.log 2>&1 || { tail -20 gpurun_out/hc_tests.log; exit 1; }
tail -1 gpurun_out/hc_tests.log
timeout -k 10 300 python bench.py --steps 20 > gpurun_out/hc_bench.json 2>/dev/null || exit 1
python3 -c "
import json; d=json.loads([l for l in open('gpurun_out/hc_bench.json') if l.startswith('{')][0]); c=d['components']
print(c['msm_2^16']['host_call_us_incl_pcie'], c['msm_2^20_host_call'], c['cpu_reference_other']['toy_prove_4_gates'])"
