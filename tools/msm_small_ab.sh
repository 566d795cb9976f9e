#!/bin/bash
# Same-session A/B of the single-launch MSM components (2^16 per launch, 2^22 one per launch) and
# the headline over the current library and plonk.c_amd/build/var/lib_*.so (tuning aid).
set -u
for rep in 1 2 3; do
  for lib in plonk.c_amd/libplonkhip.so plonk.c_amd/build/var/lib_*.so; do
    r=$(PLK_LIB=$PWD/$lib timeout -k 5 240 python bench.py --no-cpu-baseline 2>/dev/null | grep '^{') || exit 1
    echo "$lib $(echo "$r" | python3 -c 'import json,sys; d=json.load(sys.stdin); c=d["components"]; print(c["msm_2^16"]["device_us_per_msm"], c["msm_2^22_one_per_launch"]["device_us_per_msm"], d["roofline"]["frac"])')"
  done
done
