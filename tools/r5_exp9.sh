#!/bin/bash
# round-5 batch 9: the headline MSM launch with non-temporal loads (build/var/lib_msmnt.so, PLK_MSM_NT=1)
# against the default policy -- the bench headline alone (no components), alternating, three rounds
set -u
export TMPDIR=/tmp
O=gpurun_out/r5e9
mkdir -p $O
for r in 1 2 3; do
  for lib in plonk.c_amd/libplonkhip.so plonk.c_amd/build/var/lib_msmnt.so; do
    PLK_LIB=$PWD/$lib timeout -k 10 200 python3 bench.py --no-components --no-cpu-baseline --steps 50 > $O/b.json 2> $O/b.err || { echo "$lib failed"; tail $O/b.err; exit 1; }
    python3 -c "import json; d=json.loads([l for l in open('$O/b.json') if l.startswith('{')][0]); print('$(basename $lib)', d['value'], d['roofline']['frac'], d['roofline']['launch_ms_avg'])"
  done
done
echo done
