// Compile-only companion of tools/swar_probe.hip (round 2, the device-side probe): a straight-line
// sum of byte x (word & 0x00FF00FF) products -- two 16-bit lanes per multiply, bytes 0 and 2 -- is
// rewritten by ROCm 7.2's
// clang (22.0, gfx942 and gfx950, -O1 and -O3) as ONE v_dot4_u32_u8 over byte 0 of each word:
// the byte-2 lane's products are dropped.  `swar_plain` shows it; `swar_guarded` hides the mask
// behind an empty asm (prove.hip lanes02 / lanes13) and compiles to v_and + v_mad_u32_u24.
// The same miscompile gave round 2's and round 4's two-bytes-per-lane numdiv_kernel variants wrong
// t(x) bytes.
//   tools/swar_dot4_check.sh  (hipcc -S, counts v_dot4 in each kernel)
#include <hip/hip_runtime.h>
#include <stdint.h>

__global__ void swar_plain(const uint32_t* __restrict__ w, const uint8_t* __restrict__ c, uint32_t* __restrict__ out) {
  const int i = threadIdx.x;
  uint32_t e = 0;
#pragma unroll
  for (int t = 0; t < 4; t++) e += __umul24((uint32_t)c[t * 64 + i], w[t * 64 + i] & 0x00FF00FFu);
  out[i] = e;
}

__device__ __forceinline__ uint32_t lanes02(uint32_t w) {
  uint32_t m = w & 0x00FF00FFu;
  asm("" : "+v"(m));
  return m;
}

__global__ void swar_guarded(const uint32_t* __restrict__ w, const uint8_t* __restrict__ c,
                             uint32_t* __restrict__ out) {
  const int i = threadIdx.x;
  uint32_t e = 0;
#pragma unroll
  for (int t = 0; t < 4; t++) e += __umul24((uint32_t)c[t * 64 + i], lanes02(w[t * 64 + i]));
  out[i] = e;
}
