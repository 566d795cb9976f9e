# quick bench pass (tuning aid): print the components object of a short default bench run
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --steps 10 --no-cpu-baseline > gpurun_out/bc.json 2> gpurun_out/bc.err || { tail -20 gpurun_out/bc.err; exit 1; }
python3 -c "
import json; d=json.loads([l for l in open('gpurun_out/bc.json') if l.startswith('{')][0]); c=d['components']
for k in ('ntt_2^20_forward','poly_divide_zh_2^22','poly_eval_batch8_2^22','prove_2^20_gates'): print(k, c.get(k))"
