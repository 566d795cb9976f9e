#!/bin/bash
# Build a tuning variant of libplonkhip.so: one source recompiled with extra defines.
#   tools/build_var.sh NAME "-DPLK_...=..." [source: ntt_wave (default) | prove | ntt | msm | capi | polyops]
#   -> plonk.c_amd/build/var/lib_NAME.so
set -eu
SRC=${3:-ntt_wave}
cd "$(dirname "$0")/../plonk.c_amd"
make -s build/msm.o build/ntt.o build/ntt_wave.o build/capi.o build/prove.o build/polyops.o build/shards.o
mkdir -p build/var
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-result $2 \
  -c csrc/$SRC.hip -o build/var/${SRC}_$1.o
OBJS=""
for s in msm ntt ntt_wave capi prove polyops shards; do
  if [ "$s" = "$SRC" ]; then OBJS="$OBJS build/var/${SRC}_$1.o"; else OBJS="$OBJS build/$s.o"; fi
done
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 $OBJS -o build/var/lib_$1.so
