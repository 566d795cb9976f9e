// Probe (tuning aid, not part of the product): the exact lane movement of gfx950's
// v_permlane32_swap_b32 / v_permlane16_swap_b32 as the center kernel uses them (a register bit
// exchanged with lane bit 5 / lane bit 4).  Prints OK when both match that model.
//   hipcc -O3 --offload-arch=gfx950 -std=c++17 tools/permlane_probe.hip -o tools/permlane_probe
#include <hip/hip_runtime.h>
#include <stdio.h>

__global__ void k(unsigned* out) {
  const unsigned l = threadIdx.x;
  unsigned x = 1000 + l, y = 2000 + l;           // register bit 0 = 0 (x) / 1 (y)
  auto r = __builtin_amdgcn_permlane32_swap(x, y, false, false);
  out[l] = r[0];
  out[64 + l] = r[1];
  auto s = __builtin_amdgcn_permlane16_swap(x, y, false, false);
  out[128 + l] = s[0];
  out[192 + l] = s[1];
}

int main() {
  unsigned* d;
  unsigned h[256];
  if (hipMalloc(&d, sizeof h) != hipSuccess) return 1;
  hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d);
  if (hipMemcpy(h, d, sizeof h, hipMemcpyDeviceToHost) != hipSuccess) return 1;
  int bad = 0;
  for (int b = 5; b >= 4; b--) {
    const unsigned* o = h + (b == 5 ? 0 : 128);
    for (unsigned reg = 0; reg < 2; reg++)
      for (unsigned l = 0; l < 64; l++) {
        // model: element (lane l, reg) came from (lane l with bit b := reg, reg := bit b of l)
        const unsigned src_reg = (l >> b) & 1u, src_lane = (l & ~(1u << b)) | (reg << b);
        const unsigned want = (src_reg ? 2000 : 1000) + src_lane;
        if (o[reg * 64 + l] != want) {
          if (bad < 8) printf("bit %d reg %u lane %u: got %u want %u\n", b, reg, l, o[reg * 64 + l], want);
          bad++;
        }
      }
  }
  printf(bad ? "MISMATCH %d\n" : "OK\n", bad);
  return bad != 0;
}
