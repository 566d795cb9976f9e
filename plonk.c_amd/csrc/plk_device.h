// Device-side building blocks shared by the gfx950 kernels of libplonkhip.
//
//   * GF(101) group tables for the discrete-log MSM (msm.hip)
//   * BabyBear (p = 15*2^27 + 1) Montgomery arithmetic for the exact NTT poly_mul (ntt.hip)
//
// Everything here is integer work; no MFMA is involved anywhere in this library.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define PLK_WAVE 64

// Sum over the 64 lanes of a wave (every lane active), wave-uniform result: DPP row rotations
// leave each 16-lane row's sum in all its lanes, then the four row sums are read out as
// scalars.  No LDS round trips (__shfl_xor is ds_bpermute: ~6 dependent LDS latencies).
__device__ __forceinline__ uint32_t plk_wave_sum(uint32_t v) {
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x128, 0xF, 0xF, false);   // row_ror:8
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x124, 0xF, 0xF, false);   // row_ror:4
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x122, 0xF, 0xF, false);   // row_ror:2
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x121, 0xF, 0xF, false);   // row_ror:1
  return (uint32_t)__builtin_amdgcn_readlane((int)v, 0) + (uint32_t)__builtin_amdgcn_readlane((int)v, 16) +
         (uint32_t)__builtin_amdgcn_readlane((int)v, 32) + (uint32_t)__builtin_amdgcn_readlane((int)v, 48);
}

// max over the block (blockDim a multiple of 64, <= 1024); every thread gets the result.
// Called by every thread of the block (two barriers inside).
__device__ __forceinline__ uint32_t plk_block_max(uint32_t v) {
  __shared__ uint32_t red[16];
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v = max(v, (uint32_t)__shfl_xor(v, off, PLK_WAVE));
  __syncthreads();
  if ((threadIdx.x & (PLK_WAVE - 1)) == 0) red[threadIdx.x / PLK_WAVE] = v;
  __syncthreads();
  uint32_t m = 0;
  for (int w = 0; w < (int)(blockDim.x / PLK_WAVE); w++) m = max(m, red[w]);
  return m;
}

// ----------------------------------------------------------------------------------------
// BabyBear Montgomery arithmetic, R = 2^32.  Values are kept fully reduced in [0, p).
// ----------------------------------------------------------------------------------------
namespace bb {
constexpr uint32_t P = 2013265921u;          // 15 * 2^27 + 1
constexpr int TWO_ADICITY = 27;

constexpr uint32_t neg_inv_p() {             // p' = -p^{-1} mod 2^32 (Newton iteration)
  uint32_t x = 1;
  for (int i = 0; i < 5; i++) x *= 2u - P * x;
  return 0u - x;
}
constexpr uint32_t PINV = neg_inv_p();
static_assert(P * (0u - PINV) == 1u, "p * p^{-1} == 1 mod 2^32");
constexpr uint32_t R2 = (uint32_t)((((unsigned __int128)1) << 64) % P);   // R^2 mod p: mmul(x, R2) = x R

// a * b * R^-1 mod p for a < 2p, b < p (a * b < p 2^32, so REDC applies).  The 64-bit
// REDC sum t + m p < 2p 2^32, so its high word is < 2p and one unsigned min(u, u - p)
// (u - p wraps to a huge value when u < p) finishes -- 32-bit ops only after the two
// v_mad_u64_u32.
__host__ __device__ __forceinline__ uint32_t mmul(uint32_t a, uint32_t b) {
  const uint64_t t = (uint64_t)a * b;
  const uint32_t m = (uint32_t)t * PINV;
  const uint32_t u = (uint32_t)((t + (uint64_t)m * P) >> 32);
  const uint32_t v = u - P;
  return v < u ? v : u;
}
__host__ __device__ __forceinline__ uint32_t madd(uint32_t a, uint32_t b) {
  const uint32_t s = a + b;                  // a, b < p < 2^31: no wrap
  const uint32_t t = s - P;
  return t < s ? t : s;
}
__host__ __device__ __forceinline__ uint32_t msub(uint32_t a, uint32_t b) {
  const uint32_t d = a - b;                  // wraps when a < b ...
  const uint32_t e = d + P;                  // ... and then d + p < p is the answer
  return e < d ? e : d;
}
// a - b + p in [1, 2p): a valid first operand of mmul (DIF butterflies skip one reduction)
__host__ __device__ __forceinline__ uint32_t msub_lazy(uint32_t a, uint32_t b) { return a + P - b; }

// host-side helpers (plain modular arithmetic, used to build tables)
inline uint32_t hpow(uint64_t b, uint64_t e) {
  uint64_t r = 1;
  b %= P;
  while (e) {
    if (e & 1) r = r * b % P;
    b = b * b % P;
    e >>= 1;
  }
  return (uint32_t)r;
}
inline uint32_t to_mont(uint32_t x) { return (uint32_t)(((uint64_t)x << 32) % P); }
inline uint32_t from_mont(uint32_t x) { return mmul(x, 1u); }
constexpr uint32_t GENERATOR = 31;           // generates F_p^*
}  // namespace bb

// ----------------------------------------------------------------------------------------
// F29: p = 7 * 2^26 + 1 = 469762049 < 2^29, Montgomery R = 2^32, values kept LAZILY in
// [0, 8p) (bounds: ntt_wave.hip, F29 policy).  Exact for poly_mul when every convolution sum
// fits: coefficients enter as centered residues in [-8, 8], so min(la, lb) * 128 < p, i.e.
// min(la, lb) <= 3670016; larger products use BabyBear.
// ----------------------------------------------------------------------------------------
namespace f29 {
constexpr uint32_t P = 469762049u;           // 7 * 2^26 + 1
constexpr int TWO_ADICITY = 26;
constexpr uint32_t GENERATOR = 3;            // generates F_p^*
constexpr uint32_t neg_inv_p() {
  uint32_t x = 1;
  for (int i = 0; i < 5; i++) x *= 2u - P * x;
  return 0u - x;
}
constexpr uint32_t PINV = neg_inv_p();
static_assert(P * (0u - PINV) == 1u, "p * p^{-1} == 1 mod 2^32");
static_assert(8ull * P < (1ull << 32), "lazy reduction needs 8p < 2^32");
constexpr uint32_t R2 = (uint32_t)((((unsigned __int128)1) << 64) % P);
constexpr uint32_t P2 = 2 * P;

// a * b * R^-1 mod p in [0, 2p) for a * b < p 2^32 (e.g. a < 4p, b < 2p)
__host__ __device__ __forceinline__ uint32_t mmul(uint32_t a, uint32_t b) {
  const uint64_t t = (uint64_t)a * b;
  const uint32_t m = (uint32_t)t * PINV;
  return (uint32_t)((t + (uint64_t)m * P) >> 32);
}
// [0, 4p) -> [0, 2p)
__host__ __device__ __forceinline__ uint32_t red2(uint32_t x) {
  const uint32_t y = x - P2;
  return y < x ? y : x;
}
// [0, 2p) -> [0, p)
__host__ __device__ __forceinline__ uint32_t red1(uint32_t x) {
  const uint32_t y = x - P;
  return y < x ? y : x;
}
inline uint32_t hpow(uint64_t b, uint64_t e) {
  uint64_t r = 1;
  b %= P;
  while (e) {
    if (e & 1) r = r * b % P;
    b = b * b % P;
    e >>= 1;
  }
  return (uint32_t)r;
}
inline uint32_t to_mont(uint32_t x) { return (uint32_t)(((uint64_t)x << 32) % P); }
}  // namespace f29

// ----------------------------------------------------------------------------------------
// E(F101): y^2 = x^3 + 3 has 102 points and is cyclic (102 = 2*3*17).  The MSM maps every
// canonical point to its discrete log in Z/102 w.r.t. a fixed generator g0 of order 102,
// so sum c_i * P_i becomes sum c_i * log(P_i) mod 102 -- an exact group isomorphism.
//
// Per x in [0,101): one dword  Y | L << 8 | Lneg << 16
//   Y    = the smaller root y of y^2 = x^3 + 3  (0xFF: no point with this x)
//   L    = log(x, Y),  Lneg = log(x, 101 - Y) = (102 - L) mod 102
// The only point with y = 0 is the 2-torsion point (48, 0), log 51.
// Exp table: 102 canonical encodings {x, y, infinite}, index 0 = identity {0, 0, 1}.
// Both tables are built on the host at plk_init (capi.hip) from the group law itself.
// ----------------------------------------------------------------------------------------
#define PLK_GF_P 101
#define PLK_GROUP_ORDER 102
