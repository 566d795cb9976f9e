// Throughput of the modular-multiply candidates for the NTT butterflies on gfx950
// (tuning aid; build: hipcc -O3 --offload-arch=gfx950 tools/arith_bench.hip -o tools/arith_bench).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#include "../plonk.c_amd/csrc/plk_device.h"

constexpr int CH = 8;        // independent chains per thread
constexpr int ITERS = 4096;

__device__ __forceinline__ uint32_t shoup(uint32_t x, uint32_t w, uint32_t wq) {
  const uint32_t q = __umulhi(x, wq);
  const uint32_t r = x * w - q * bb::P;
  return r >= bb::P ? r - bb::P : r;
}

template <int MODE>
__global__ void k_arith(uint32_t* out, uint32_t seed) {
  uint32_t v[CH];
  const uint32_t w = 0x12345678u % bb::P, wq = (uint32_t)(((uint64_t)w << 32) / bb::P);
#pragma unroll
  for (int i = 0; i < CH; i++) v[i] = (seed + threadIdx.x * 7 + i * 13) % bb::P;
  for (int it = 0; it < ITERS; it++) {
#pragma unroll
    for (int i = 0; i < CH; i++) {
      if (MODE == 0) v[i] = bb::mmul(v[i], w);
      else if (MODE == 1) v[i] = shoup(v[i], w, wq);
      else if (MODE == 2) v[i] = bb::madd(v[i], w);
      else if (MODE == 3) v[i] = v[i] * w + 1u;                  // v_mul_lo_u32 (+add)
      else if (MODE == 4) v[i] = __umulhi(v[i], w) ^ v[i];       // v_mul_hi_u32
      else if (MODE == 5) v[i] = __umul24(v[i], w) + 1u;         // v_mul_u32_u24
    }
  }
  uint32_t s = 0;
#pragma unroll
  for (int i = 0; i < CH; i++) s ^= v[i];
  if (s == 0x9e3779b9u) out[0] = s;
}

__global__ void k_fma64(double* out, double seed) {
  double v[CH];
#pragma unroll
  for (int i = 0; i < CH; i++) v[i] = seed + threadIdx.x + i;
  for (int it = 0; it < ITERS; it++) {
#pragma unroll
    for (int i = 0; i < CH; i++) v[i] = fma(v[i], 0.999999, 1e-9);
  }
  double s = 0;
#pragma unroll
  for (int i = 0; i < CH; i++) s += v[i];
  if (s == 12345.0) out[0] = s;
}

template <typename F>
static double time_ms(F f) {
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  f();
  hipDeviceSynchronize();
  hipEventRecord(a);
  for (int i = 0; i < 5; i++) f();
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms;
  hipEventElapsedTime(&ms, a, b);
  return ms / 5;
}

int main() {
  uint32_t* d;
  hipMalloc(&d, 64);
  const int blocks = 256 * 8, threads = 256;
  const double ops = (double)blocks * threads * CH * ITERS;
  const char* names[] = {"montgomery_mmul", "shoup_mul", "madd", "mul_lo_u32", "mul_hi_u32", "mul_u32_u24"};
  double ms[6];
  ms[0] = time_ms([&] { hipLaunchKernelGGL(k_arith<0>, dim3(blocks), dim3(threads), 0, 0, d, 1u); });
  ms[1] = time_ms([&] { hipLaunchKernelGGL(k_arith<1>, dim3(blocks), dim3(threads), 0, 0, d, 1u); });
  ms[2] = time_ms([&] { hipLaunchKernelGGL(k_arith<2>, dim3(blocks), dim3(threads), 0, 0, d, 1u); });
  ms[3] = time_ms([&] { hipLaunchKernelGGL(k_arith<3>, dim3(blocks), dim3(threads), 0, 0, d, 1u); });
  ms[4] = time_ms([&] { hipLaunchKernelGGL(k_arith<4>, dim3(blocks), dim3(threads), 0, 0, d, 1u); });
  ms[5] = time_ms([&] { hipLaunchKernelGGL(k_arith<5>, dim3(blocks), dim3(threads), 0, 0, d, 1u); });
  const double fms = time_ms([&] { hipLaunchKernelGGL(k_fma64, dim3(blocks), dim3(threads), 0, 0, (double*)d, 1.0); });
  printf("{");
  for (int i = 0; i < 6; i++) printf("\"%s_Gop_s\": %.1f, ", names[i], ops / (ms[i] * 1e-3) / 1e9);
  printf("\"fma_f64_Gop_s\": %.1f}\n", ops / (fms * 1e-3) / 1e9);
  return 0;
}
