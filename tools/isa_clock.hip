// VALU issue rate in SHADER CYCLES (s_memtime), per SIMD, vs waves per SIMD (tuning aid):
// 256 threads per block, B blocks per CU all resident (B*4 waves per CU = B per SIMD); each
// wave runs 8 independent chains of one instruction.  Prints cycles per wave instruction
// per SIMD = elapsed cycles of a wave / (instructions per wave * waves per SIMD).
//   hipcc -O3 --offload-arch=gfx950 tools/isa_clock.hip -o tools/isa_clock
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

constexpr int ITERS = 4096;

template <int OP>
__global__ __launch_bounds__(256) void k(uint64_t* cyc, uint32_t* out, uint32_t seed) {
  uint32_t a[8];
  uint64_t w[8];
#pragma unroll
  for (int i = 0; i < 8; i++) { a[i] = seed + threadIdx.x * 3 + i; w[i] = a[i] * 7ull; }
  const uint32_t m = 0x12345679u;
  __syncthreads();
  const uint64_t t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < ITERS; it++) {
#pragma unroll
    for (int i = 0; i < 8; i++) {
      if (OP == 0) asm volatile("v_add_u32 %0, %0, %1" : "+v"(a[i]) : "s"(m));
      if (OP == 1) asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(a[i]) : "s"(m));
      if (OP == 2) asm volatile("v_mad_u64_u32 %0, vcc, %1, %2, %0" : "+v"(w[i]) : "v"(a[i]), "s"(m) : "vcc");
      if (OP == 3) asm volatile("v_min_u32 %0, %0, %1" : "+v"(a[i]) : "v"(a[(i + 1) & 7]));
    }
  }
  const uint64_t t1 = __builtin_amdgcn_s_memtime();
  uint32_t s = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) s ^= a[i] ^ (uint32_t)w[i];
  if (s == 0x9e3779b9u) out[0] = s;
  if (threadIdx.x % 64 == 0) cyc[blockIdx.x * 4 + threadIdx.x / 64] = t1 - t0;
}

template <int OP>
void run(const char* name, uint64_t* d, uint32_t* o, int cus) {
  for (int per_simd = 1; per_simd <= 8; per_simd *= 2) {
    const int blocks = cus * per_simd;   // 4 waves per block: per_simd blocks per CU
    hipLaunchKernelGGL(k<OP>, dim3(blocks), dim3(256), 0, 0, d, o, 1u);
    hipLaunchKernelGGL(k<OP>, dim3(blocks), dim3(256), 0, 0, d, o, 1u);
    (void)hipDeviceSynchronize();
    static uint64_t h[256 * 8 * 4];
    (void)hipMemcpy(h, d, sizeof(uint64_t) * blocks * 4, hipMemcpyDeviceToHost);
    double sum = 0;
    uint64_t mx = 0;
    for (int i = 0; i < blocks * 4; i++) { sum += h[i]; mx = h[i] > mx ? h[i] : mx; }
    const double inst = (double)ITERS * 8;
    printf("%-14s waves/SIMD %d: avg %.2f max %.2f cycles per wave-instruction per SIMD (memtime)\n", name, per_simd,
           sum / (blocks * 4) / inst / per_simd, mx / inst / per_simd);
  }
}

int main() {
  uint64_t* d;
  uint32_t* o;
  (void)hipMalloc(&d, sizeof(uint64_t) * 256 * 8 * 4);
  (void)hipMalloc(&o, 64);
  hipDeviceProp_t p;
  (void)hipGetDeviceProperties(&p, 0);
  printf("CUs %d, clock %d kHz\n", p.multiProcessorCount, p.clockRate);
  run<0>("v_add_u32", d, o, p.multiProcessorCount);
  run<1>("v_mul_lo_u32", d, o, p.multiProcessorCount);
  run<2>("v_mad_u64_u32", d, o, p.multiProcessorCount);
  run<3>("v_min_u32", d, o, p.multiProcessorCount);
  return 0;
}
