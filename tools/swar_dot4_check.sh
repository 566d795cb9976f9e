#!/bin/bash
# Compile tools/swar_dot4_repro.hip for gfx950 and print, per kernel, its v_dot4_u32_u8 and
# 0xff00ff-mask counts: "swar_plain dot4=1 mask=0" is the miscompile, "swar_guarded dot4=0 mask=4"
# the guarded form prove.hip uses.  CPU only (hipcc -S).
set -eu
cd "$(dirname "$0")"
out=$(mktemp -d)
/opt/rocm/bin/hipcc -O3 --offload-arch=gfx950 --cuda-device-only -S swar_dot4_repro.hip -o "$out/r.s" 2>/dev/null
for k in swar_plain swar_guarded; do
  body=$(awk -v K="$k" '$0 ~ "^_Z[0-9]+"K".*:" {f=1} f && /s_endpgm/ {f=0} f' "$out/r.s")
  echo "$k dot4=$(grep -c v_dot4 <<<"$body" || true) mask=$(grep -c 0xff00ff <<<"$body" || true)"
done
rm -rf "$out"
