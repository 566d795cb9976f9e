#!/bin/bash
# Same-session A/B of the MSM headline (bench.py, no components / CPU baseline) over the
# current library and plonk.c_amd/build/var/lib_*.so (tuning aid).
set -u
for rep in 1 2 3; do
  for lib in plonk.c_amd/libplonkhip.so plonk.c_amd/build/var/lib_*.so; do
    r=$(PLK_LIB=$PWD/$lib timeout -k 5 180 python bench.py --no-components --no-cpu-baseline 2>/dev/null | grep '^{') || exit 1
    echo "$lib $(echo "$r" | python3 -c 'import json,sys; d=json.load(sys.stdin); print(d["value"], d["roofline"]["frac"], d["roofline"]["launch_ms_avg"])')"
  done
done
