#!/bin/bash
# Build a tuning variant of libplonkhip.so: ntt_wave.hip recompiled with extra defines.
#   tools/build_var.sh NAME "-DPLK_NTT_DIAG=1 ..."  ->  plonk.c_amd/build/var/lib_NAME.so
set -eu
cd "$(dirname "$0")/../plonk.c_amd"
make -s build/msm.o build/ntt.o build/capi.o build/prove.o
mkdir -p build/var
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-result $2 \
  -c csrc/ntt_wave.hip -o build/var/ntt_wave_$1.o
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 build/msm.o build/ntt.o build/capi.o build/prove.o \
  build/var/ntt_wave_$1.o -o build/var/lib_$1.so
