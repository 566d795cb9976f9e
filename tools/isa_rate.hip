// Issue-rate probe for the integer multiplies of the NTT butterflies on gfx950 (tuning aid):
// 8 independent dependency chains per lane of one instruction, inline asm so nothing folds.
//   hipcc -O3 --offload-arch=gfx950 tools/isa_rate.hip -o tools/isa_rate
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

constexpr int ITERS = 2048;

template <int OP>
__global__ __launch_bounds__(256) void k(uint32_t* out, uint32_t seed) {
  uint32_t a[8];
  uint64_t w[8];
#pragma unroll
  for (int i = 0; i < 8; i++) { a[i] = seed + threadIdx.x * 3 + i; w[i] = a[i] * 7ull; }
  const uint32_t m = 0x12345679u;
  for (int it = 0; it < ITERS; it++) {
#pragma unroll
    for (int i = 0; i < 8; i++) {
      if (OP == 0) asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(a[i]) : "s"(m));
      if (OP == 1) asm volatile("v_mul_hi_u32 %0, %0, %1" : "+v"(a[i]) : "s"(m));
      if (OP == 2) asm volatile("v_mad_u64_u32 %0, vcc, %1, %2, %0" : "+v"(w[i]) : "v"(a[i]), "s"(m) : "vcc");
      if (OP == 3) asm volatile("v_add_u32 %0, %0, %1" : "+v"(a[i]) : "s"(m));
      if (OP == 4) asm volatile("v_mul_u32_u24 %0, %0, %1" : "+v"(a[i]) : "s"(m));
      if (OP == 5) asm volatile("v_mul_f32 %0, %0, %1" : "+v"(a[i]) : "s"(m));
      if (OP == 6) asm volatile("v_mul_f64 %0, %0, %1" : "+v"(w[i]) : "v"(w[i]));
      if (OP == 7) asm volatile("v_cvt_f64_u32 %0, %1" : "=v"(w[i]) : "v"(a[i]));
      // gfx950 cross-lane swaps (the lane-swap center kernel): register pairs (i, i ^ 1), so
      // 8 instructions per iteration as for the others
      if (OP == 8) asm volatile("v_permlane32_swap_b32 %0, %1" : "+v"(a[i]), "+v"(a[i ^ 1]));
      if (OP == 9) asm volatile("v_permlane16_swap_b32 %0, %1" : "+v"(a[i]), "+v"(a[i ^ 1]));
    }
  }
  uint32_t s = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) s ^= a[i] ^ (uint32_t)w[i];
  if (s == 0x9e3779b9u) out[0] = s;
}

template <int OP>
double run(uint32_t* d) {
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  const int blocks = 256 * 16, threads = 256;
  hipLaunchKernelGGL(k<OP>, dim3(blocks), dim3(threads), 0, 0, d, 1u);
  (void)hipEventRecord(e0);
  hipLaunchKernelGGL(k<OP>, dim3(blocks), dim3(threads), 0, 0, d, 1u);
  (void)hipEventRecord(e1);
  (void)hipEventSynchronize(e1);
  float ms;
  (void)hipEventElapsedTime(&ms, e0, e1);
  const double insts = (double)blocks * threads / 64 * ITERS * 8;   // wave instructions
  // cycles per wave instruction per SIMD at 2.4 GHz: 1024 SIMDs
  return ms * 1e-3 * 2.4e9 * 1024 / insts;
}

int main() {
  uint32_t* d;
  (void)hipMalloc(&d, 64);
  printf("cycles per wave64 instruction per SIMD (2.4 GHz assumed):\n");
  printf("v_mul_lo_u32   %.2f\n", run<0>(d));
  printf("v_mul_hi_u32   %.2f\n", run<1>(d));
  printf("v_mad_u64_u32  %.2f\n", run<2>(d));
  printf("v_add_u32      %.2f\n", run<3>(d));
  printf("v_mul_u32_u24  %.2f\n", run<4>(d));
  printf("v_mul_f32      %.2f\n", run<5>(d));
  printf("v_mul_f64      %.2f\n", run<6>(d));
  printf("v_cvt_f64_u32  %.2f\n", run<7>(d));
  printf("v_permlane32_swap_b32  %.2f\n", run<8>(d));
  printf("v_permlane16_swap_b32  %.2f\n", run<9>(d));
  return 0;
}
