// Butterfly-throughput peak (measurement aid, not part of the product): the chip-wide rate of the
// NTT engine's radix-2 butterflies with the operands in registers -- no memory, no LDS -- at
// full occupancy (two 1024-thread blocks per CU).  This is the compute roof the NTT kernels are
// priced against (tools/ntt_roofline.py): a pass kernel's butterflies / its duration / this rate.
// The butterflies are the engine's own formulas (ntt_wave.hip F29 / FBB policies, restated from
// plk_device.h's primitives): F29 lazy DIF (two v_mad_u64_u32 + REDC, sum reduced every other
// stage) and DIT, BabyBear DIF / DIT (fully reduced), and a bare v_add_u32 chain for reference.
// Also measured: Shoup multiplies (a second twiddle word w' = floor(w 2^32 / p), one mul_hi +
// two mul_lo per product) as a candidate for the F29 butterflies -- 4715 / 4678 Gbfly/s against
// Montgomery's 5873 / 5358 (DIF / DIT), so the engine keeps Montgomery.
//
//   hipcc -O3 --offload-arch=gfx950 -std=c++17 -I plonk.c_amd/csrc tools/bfly_peak.hip -o tools/bfly_peak
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#include "plk_device.h"

#define CK(x)                                                         \
  do {                                                                \
    hipError_t e = (x);                                               \
    if (e != hipSuccess) {                                            \
      printf("%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e)); \
      return 1;                                                       \
    }                                                                 \
  } while (0)

namespace {
__device__ __forceinline__ uint32_t red4(uint32_t x) {
  const uint32_t y = x - 2 * f29::P2;
  return y < x ? y : x;
}
__device__ __forceinline__ void f29_dif(uint32_t& u, uint32_t& x, uint32_t w, bool red) {
  const uint32_t a = u, b = x;
  const uint64_t t = (uint64_t)a * w + (uint64_t)b * (f29::P - w);
  const uint32_t m = (uint32_t)t * f29::PINV;
  x = (uint32_t)((t + (uint64_t)m * f29::P) >> 32);
  const uint32_t s = a + b;
  u = red ? red4(s) : s;
}
__device__ __forceinline__ void f29_dit(uint32_t& u, uint32_t& x, uint32_t w, bool red) {
  const uint32_t xw = f29::mmul(x, w);
  const uint32_t a = red ? red4(u) : u;
  u = a + xw;
  x = a + f29::P2 - xw;
}
__device__ __forceinline__ void bb_dif(uint32_t& u, uint32_t& x, uint32_t w, bool) {
  const uint32_t a = u, b = x;
  u = bb::madd(a, b);
  x = bb::mmul(bb::msub_lazy(a, b), w);
}
__device__ __forceinline__ void bb_dit(uint32_t& u, uint32_t& x, uint32_t w, bool) {
  const uint32_t xw = bb::mmul(x, w), a = u;
  u = bb::madd(a, xw);
  x = bb::msub(a, xw);
}

// Shoup forms (candidates): x w mod p = x w - floor(x w' / 2^32) p in [0, 2p) for any u32 x,
// w' = floor(w 2^32 / p) (a second twiddle word)
__device__ __forceinline__ uint32_t shoup(uint32_t x, uint32_t w, uint32_t wp, uint32_t p) {
  const uint32_t q = __umulhi(x, wp);
  return x * w - q * p;
}
__device__ __forceinline__ void f29s_dif(uint32_t& u, uint32_t& x, uint32_t w, uint32_t wp, bool red) {
  const uint32_t a = u, b = x;                 // < 4p
  x = shoup(a + 4 * f29::P - b, w, wp, f29::P);   // < 2p
  const uint32_t s = a + b;
  u = red ? red4(s) : s;
}
__device__ __forceinline__ void f29s_dit(uint32_t& u, uint32_t& x, uint32_t w, uint32_t wp, bool red) {
  const uint32_t xw = shoup(x, w, wp, f29::P);
  const uint32_t a = red ? red4(u) : u;
  u = a + xw;
  x = a + f29::P2 - xw;
}

// 8 values per thread, 3 stages of 4 butterflies per iteration (a radix-2^3 round in registers,
// the engine's R = 3 shape), twiddles in registers (distinct per stage)
template <int KIND>
__global__ __launch_bounds__(1024, 8) void k_bfly(uint32_t* out, int iters, uint32_t seed) {
  uint32_t v[8];
  const uint32_t t = blockIdx.x * 1024 + threadIdx.x;
#pragma unroll
  for (int k = 0; k < 8; k++) v[k] = (t * 2654435761u + k * 40503u + seed) % f29::P;
  const uint32_t w0 = (seed * 7u + 3u) % f29::P, w1 = (seed * 11u + 5u) % f29::P, w2 = (seed * 13u + 9u) % f29::P;
  const uint32_t q0 = (uint32_t)(((uint64_t)w0 << 32) / f29::P), q1 = (uint32_t)(((uint64_t)w1 << 32) / f29::P),
                 q2 = (uint32_t)(((uint64_t)w2 << 32) / f29::P);
  for (int it = 0; it < iters; it++) {
#pragma unroll
    for (int s = 2; s >= 0; s--) {
      const uint32_t w = s == 2 ? w0 : (s == 1 ? w1 : w2);
      const uint32_t wq = s == 2 ? q0 : (s == 1 ? q1 : q2);
#pragma unroll
      for (int k = 0; k < 8; k++) {
        if (k & (1 << s)) continue;
        uint32_t& a = v[k];
        uint32_t& b = v[k | (1 << s)];
        if (KIND == 0) f29_dif(a, b, w, s != 1);
        else if (KIND == 1) f29_dit(a, b, w, s != 1);
        else if (KIND == 2) bb_dif(a, b, w, false);
        else if (KIND == 3) bb_dit(a, b, w, false);
        else if (KIND == 5) f29s_dif(a, b, w, wq, s != 1);
        else if (KIND == 6) f29s_dit(a, b, w, wq, s != 1);
        else {
          a += b;
          b += a;
        }
      }
    }
  }
  uint32_t x = 0;
#pragma unroll
  for (int k = 0; k < 8; k++) x ^= v[k];
  if (x == 0x12345678u) out[t] = x;
}
}  // namespace

int main() {
  int dev = 0, cus = 0;
  CK(hipGetDevice(&dev));
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
  uint32_t* out;
  CK(hipMalloc(&out, 4u << 20));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  const int blocks = 2 * cus, iters = 4096;
  const char* names[] = {"f29_dif", "f29_dit", "bb_dif", "bb_dit", "add_u32_pair", "f29_shoup_dif", "f29_shoup_dit"};
  printf("{\"cus\": %d, \"blocks\": %d, \"threads\": 1024", cus, blocks);
  for (int kind = 0; kind < 7; kind++) {
    auto launch = [&](int it) {
      switch (kind) {
        case 0: hipLaunchKernelGGL(k_bfly<0>, dim3(blocks), dim3(1024), 0, 0, out, it, 7u); break;
        case 1: hipLaunchKernelGGL(k_bfly<1>, dim3(blocks), dim3(1024), 0, 0, out, it, 7u); break;
        case 2: hipLaunchKernelGGL(k_bfly<2>, dim3(blocks), dim3(1024), 0, 0, out, it, 7u); break;
        case 3: hipLaunchKernelGGL(k_bfly<3>, dim3(blocks), dim3(1024), 0, 0, out, it, 7u); break;
        case 4: hipLaunchKernelGGL(k_bfly<4>, dim3(blocks), dim3(1024), 0, 0, out, it, 7u); break;
        case 5: hipLaunchKernelGGL(k_bfly<5>, dim3(blocks), dim3(1024), 0, 0, out, it, 7u); break;
        default: hipLaunchKernelGGL(k_bfly<6>, dim3(blocks), dim3(1024), 0, 0, out, it, 7u); break;
      }
    };
    launch(16);
    CK(hipDeviceSynchronize());
    float best = 1e30f;
    for (int r = 0; r < 5; r++) {
      CK(hipEventRecord(a, 0));
      launch(iters);
      CK(hipEventRecord(b, 0));
      CK(hipEventSynchronize(b));
      float ms;
      CK(hipEventElapsedTime(&ms, a, b));
      if (ms < best) best = ms;
    }
    CK(hipGetLastError());
    const double bfly = (double)blocks * 1024 * iters * 12;   // 3 stages x 4 butterflies per iteration
    printf(", \"%s_Gbfly_s\": %.1f", names[kind], bfly / (best * 1e-3) / 1e9);
  }
  printf("}\n");
  return 0;
}
