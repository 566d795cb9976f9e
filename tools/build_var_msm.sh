#!/bin/bash
# Build a tuning variant of libplonkhip.so with msm.hip recompiled with extra defines.
#   tools/build_var_msm.sh NAME "-DPLK_MSM_...=..."  ->  plonk.c_amd/build/var/lib_NAME.so
set -eu
cd "$(dirname "$0")/../plonk.c_amd"
make -s build/ntt.o build/ntt_wave.o build/capi.o build/prove.o
mkdir -p build/var
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-result $2 -c csrc/msm.hip -o build/var/msm_$1.o
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 build/var/msm_$1.o build/ntt.o build/ntt_wave.o build/capi.o \
  build/prove.o -o build/var/lib_$1.so
