// Device-resident PLONK prover (reference plonk_prove, src/plonk.h:223-656) on gfx950.
//
// Everything between the circuit upload and the 34 proof bytes runs on one stream with no
// host round trip: the 17 poly_mul of the prover go through the NTT path (ntt.hip /
// ntt_wave.hip), the poly_add / poly_sub / poly_scale / poly_add_hf chains are fused into
// one "lincomb" kernel each, poly_eval is a batched reduction, poly_divide by Z_H = x^m + c
// is a strided chain walk and by a linear factor a suffix scan, and the 9 KZG commitments
// (srs_eval_at_s) are ONE batched discrete-log MSM launch over a [9][stride] scalar arena.
// Scalars derived from evaluations (a_z, b_z, ... and the r(x) / w(x) coefficients) live in
// a small device "scalar file" written by single-thread kernels, so no kernel waits on
// the host.
//
// Polynomials are carried at upper-bound lengths (untrimmed).  Every reference operation
// used here is value-identical under zero extension (poly_add/sub/scale/mul, poly_eval,
// poly_divide by a trimmed divisor, poly_slice of the quotient), so the commitments and
// evaluations -- hence the proof bytes -- equal the reference's; the trimmed lengths that
// decide the reference's error exits (SRS too short, t(x) too short to slice, non-zero
// remainders, failed asserts) are computed on the device and checked once at the end.
#include <stdio.h>
#include <stdlib.h>
#include <sched.h>
#include <string.h>

#include <algorithm>
#include <initializer_list>
#include <tuple>
#include <utility>
#include <string>
#include <vector>

#include "plk_device.h"
#include "plk_internal.h"
#include "plk_msm_finish.h"

// Diagnostic builds only (plonk.c_amd/Makefile `diag`): 1 drops plk_prover_chains_dev's ordering of
// `done` behind the chains, 2 drops plk_prover_rounds_ext_dev's wait for `ready` -- the hand-off
// orderings tests/test_split_streams_gpu.py must catch.  0 in the library.
#ifndef PLK_DIAG_DROP_HANDOFF
#define PLK_DIAG_DROP_HANDOFF 0
#endif

namespace {

constexpr uint32_t HFP = 17;

// ------------------------------------------------------------------ scalar file layout
enum Slot : int {
  S_ZERO = 0, S_ONE, S_NEG1,
  S_ALPHA, S_BETA, S_GAMMA, S_Z, S_V,
  S_OMEGA, S_K1, S_K2,
  S_BK1, S_BK2, S_ALPHA2, S_ZN2, S_Z2N4, S_V2, S_V3, S_V4, S_V5, S_V6, S_NEGZ, S_ZOMEGA,
  // evaluations (round 4)
  S_AZ = 32, S_BZ, S_CZ, S_S1Z, S_S2Z, S_TZ, S_ZWZ, S_L1Z, S_RZ, S_ACCW,
  // derived from evaluations
  S_AB = 48, S_R24, S_BZW, S_R3, S_W0, S_NEGZWZ, S_R3B,
  // small constant polynomials (blinding factors), 4-byte aligned
  P_BLA = 64, P_BLB = 68, P_BLC = 72, P_BLZ = 76,
  // evaluations at z of r(x)'s terms (r_z without materialising r(x) for it), and w_z(x)'s
  // coefficients of those terms (v times r(x)'s scalars)
  S_QMZ = 80, S_QLZ, S_QRZ, S_QOZ, S_ZXZ, S_P3Z,
  S_VAB = 88, S_VAZ, S_VBZ, S_VCZ, S_VR24, S_VR3B,
  NSLOT = 128
};

// status words (device -> host once per proof)
enum Stat : int {
  ST_LEN0 = 0,          // trimmed lengths of the 9 committed polynomials
  ST_TXLEN = 9,         // trimmed length of t(x)
  ST_REM_T = 10,        // t(x) numerator mod Z_H != 0
  ST_REM_W1 = 11,       // w_z remainder != 0
  ST_REM_W2 = 12,       // w_z_omega remainder != 0
  ST_GATE = 13,         // 1 + first unsatisfied gate
  ST_COPY = 14,         // 1 + first invalid copy constraint
  ST_ACC = 15,          // acc_x(omega^n) (must be 1)
  NSTAT = 16
};

__device__ __forceinline__ uint32_t hneg(uint32_t a) { return a ? HFP - a : 0; }
// x mod 17 for x < 69632 by 24-bit multiplies (full rate; `% 17` on a u32 takes a quarter-rate
// multiply-high): 61681 = (2^20 + 1) / 17, so floor(x 61681 / 2^20) = floor(x / 17) for x < 2^20,
// and x 61681 < 2^32 (checked on the host for every x < 69632).  Every call site's bound is noted.
__device__ __forceinline__ uint32_t hmod(uint32_t x) { return x - 17u * (__umul24(x, 61681u) >> 20); }
__device__ __forceinline__ uint32_t hpow_d(uint32_t b, uint64_t e) {
  uint32_t r = 1;
  b %= HFP;
  while (e) {
    if (e & 1) r = r * b % HFP;
    b = b * b % HFP;
    e >>= 1;
  }
  return r;
}
__device__ __forceinline__ uint32_t hinv(uint32_t a) { return hpow_d(a, HFP - 2); }   // inv(0) = 0 (hf.h LUT)

// ------------------------------------------------------------------ lincomb
// out[i] = S[scale] * (sum_t S[slot_t] * p_t[i] + [i==0] S[c0] + [i==1] S[c1]) mod 17,
// optionally times S[twist]^i.  Covers poly_add/sub/scale/add_hf chains (src/poly.h:67-104,
// :179-197) and the z(omega x) twist (src/plonk.h:459-463).
constexpr int LC_MAX = 16;
struct LcArgs {
  const uint8_t* p[LC_MAX];
  uint64_t len[LC_MAX];
  int slot[LC_MAX];
  int nt;
  int c0, c1;       // constant slots added at coefficients 0 / 1 (-1: none)
  int scale;        // slot of the outer factor
  int twist;        // slot x: multiply coefficient i by x^i (-1: none)
  uint8_t* out;
  uint64_t out_len;
};

__global__ __launch_bounds__(256) void lincomb_kernel(LcArgs a, const uint8_t* __restrict__ S) {
  uint32_t cf[LC_MAX];
#pragma unroll
  for (int t = 0; t < LC_MAX; t++) cf[t] = t < a.nt ? S[a.slot[t]] : 0u;
  const uint32_t sc = S[a.scale];
  const uint32_t c0 = a.c0 >= 0 ? S[a.c0] : 0u, c1 = a.c1 >= 0 ? S[a.c1] : 0u;
  uint32_t tw[16];
  const uint32_t x = a.twist >= 0 ? S[a.twist] : 1u;
  tw[0] = 1;
#pragma unroll
  for (int j = 1; j < 16; j++) tw[j] = tw[j - 1] * x % HFP;
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < a.out_len; i += stride) {
    uint32_t acc = i == 0 ? c0 : (i == 1 ? c1 : 0u);
#pragma unroll
    for (int t = 0; t < LC_MAX; t++)
      if (t < a.nt && i < a.len[t]) acc += cf[t] * a.p[t][i];
    uint32_t v = acc % HFP * sc % HFP;
    if (a.twist >= 0) v = v * (i == 0 ? 1u : (x == 0 ? 0u : tw[i & 15])) % HFP;
    a.out[i] = (uint8_t)v;
  }
}

// 16 coefficients per thread and iteration (uint4 loads / stores); every pointer 16-byte
// aligned (checked on the host, else lincomb_kernel).
__device__ __forceinline__ void load16(const uint8_t* p, uint64_t len, uint64_t i, uint32_t (&w)[4]) {
  if (i + 16 <= len) {
    const uint4 q = *reinterpret_cast<const uint4*>(p + i);
    w[0] = q.x; w[1] = q.y; w[2] = q.z; w[3] = q.w;
    return;
  }
  w[0] = w[1] = w[2] = w[3] = 0;
#pragma unroll
  for (int k = 0; k < 16; k++)
    if (i + k < len) w[k >> 2] |= (uint32_t)p[i + k] << (8 * (k & 3));
}

// p readable in whole 16-byte chunks up to len (16-byte aligned): one unconditional uint4
// load at a clamped address, bytes past len masked
__device__ __forceinline__ void load16_masked(const uint8_t* p, uint64_t len, uint64_t i, uint32_t (&w)[4]) {
  const bool in = i < len;
  const uint4 q = *reinterpret_cast<const uint4*>(p + (in ? i : 0));
  const uint32_t v[4] = {q.x, q.y, q.z, q.w};
#pragma unroll
  for (int k = 0; k < 4; k++) {
    const int64_t cnt = in ? (int64_t)len - (int64_t)(i + 4 * k) : 0;   // valid bytes in word k
    w[k] = cnt >= 4 ? v[k] : (cnt <= 0 ? 0u : v[k] & ((1u << (8 * cnt)) - 1u));
  }
}
__global__ __launch_bounds__(256) void lincomb16_kernel(LcArgs a, const uint8_t* __restrict__ S) {
  uint32_t cf[LC_MAX];
#pragma unroll
  for (int t = 0; t < LC_MAX; t++) cf[t] = t < a.nt ? S[a.slot[t]] : 0u;
  const uint32_t sc = S[a.scale];
  const uint32_t c0 = a.c0 >= 0 ? S[a.c0] : 0u, c1 = a.c1 >= 0 ? S[a.c1] : 0u;
  const uint32_t x = a.twist >= 0 ? S[a.twist] : 1u;
  uint32_t tw[16];   // x^k; x^i = 1 for i = 0 mod 16 when x != 0
  tw[0] = 1;
#pragma unroll
  for (int k = 1; k < 16; k++) tw[k] = tw[k - 1] * x % HFP;
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x * 16;
  for (uint64_t i = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) * 16; i < a.out_len; i += stride) {
    uint32_t acc[16];
#pragma unroll
    for (int k = 0; k < 16; k++) acc[k] = 0;
    if (i == 0) { acc[0] = c0; acc[1] = c1; }
#pragma unroll
    for (int t = 0; t < LC_MAX; t++) {
      if (t < a.nt && i < a.len[t]) {
        uint32_t w[4];
        load16(a.p[t], a.len[t], i, w);
#pragma unroll
        for (int k = 0; k < 16; k++) acc[k] += cf[t] * ((w[k >> 2] >> (8 * (k & 3))) & 0xFFu);
      }
    }
    uint32_t o[4] = {0, 0, 0, 0};
#pragma unroll
    for (int k = 0; k < 16; k++) {
      uint32_t v = hmod(hmod(acc[k]) * sc);   // (acc <= 16 terms x 16 x 255 + 32 < 69632)
      if (a.twist >= 0) v = hmod(v * (x == 0 ? (i + k == 0 ? 1u : 0u) : tw[k]));
      o[k >> 2] |= v << (8 * (k & 3));
    }
    if (i + 16 <= a.out_len) {
      *reinterpret_cast<uint4*>(a.out + i) = make_uint4(o[0], o[1], o[2], o[3]);
    } else {
#pragma unroll
      for (int k = 0; k < 16; k++)
        if (i + k < a.out_len) a.out[i + k] = (uint8_t)(o[k >> 2] >> (8 * (k & 3)));
    }
  }
}

// Rounds 1-3 preparation in ONE launch (every step is elementwise up to a shift of 2):
//   a_x = (b2 + b1 x) Z_H + f_a, b_x, c_x (src/plonk.h:280-296), z_x = (b9 + b8 x + b7 x^2) Z_H
//   + acc_x (:371-377), then round 3's linear factors alpha (a + beta x + gamma), b + beta k1 x +
//   gamma, c + beta k2 x + gamma, alpha (a + beta s1 + gamma), b + beta s2 + gamma, c + beta s3 +
//   gamma, z(omega x), alpha^2 (z - 1) (:409-489).  Same bytes as the 4 blinding poly_muls and 3
//   lincomb launches it replaces (the first kernels of a proof are host-launch bound).
struct SlotFile {
  uint8_t b[NSLOT];
};
struct PrepArgs {
  const uint8_t *zh, *fa, *fb, *fc, *acc, *s1, *s2, *s3;
  uint64_t lz, n, la, lzx;
  uint8_t *cA, *cB, *cC, *cZ, *A2, *B2, *C2, *A3, *B3, *C3, *ZW, *Z1;
};
// 4 coefficients per thread (dword loads / stores): a 2^20-gate proof has 2^18 threads, four
// waves per SIMD to overlap the loads (16 per thread left one wave per SIMD: 18 us)
__device__ __forceinline__ uint32_t load4(const uint8_t* p, uint64_t len, uint64_t i) {
  if (i + 4 <= len) return *reinterpret_cast<const uint32_t*>(p + i);
  uint32_t w = 0;
#pragma unroll
  for (int k = 0; k < 4; k++)
    if (i + k < len) w |= (uint32_t)p[i + k] << (8 * k);
  return w;
}
__device__ __forceinline__ void store4(uint8_t* out, uint64_t len, uint64_t i, uint32_t w) {
  if (i + 4 <= len) {
    *reinterpret_cast<uint32_t*>(out + i) = w;
  } else {
#pragma unroll
    for (int k = 0; k < 4; k++)
      if (i + k < len) out[i + k] = (uint8_t)(w >> (8 * k));
  }
}
// The scalar file comes in as an argument: block 0 also stores it to the device copy the later
// kernels read and clears status words [0, st1) (scalars_init_kernel's work: one launch fewer).
__global__ __launch_bounds__(256) void prep_kernel(PrepArgs a, const SlotFile f, uint8_t* __restrict__ Sd,
                                                   uint32_t* __restrict__ stat, int st1) {
  const uint8_t* S = f.b;
  if (blockIdx.x == 0) {
    if (threadIdx.x < NSLOT) Sd[threadIdx.x] = f.b[threadIdx.x];
    if ((int)threadIdx.x < st1) stat[threadIdx.x] = 0;
  }
  const uint32_t al = S[S_ALPHA], be = S[S_BETA], ga = S[S_GAMMA], bk1 = S[S_BK1], bk2 = S[S_BK2];
  const uint32_t al2 = S[S_ALPHA2], om = S[S_OMEGA];
  const uint32_t ba0 = S[P_BLA], ba1 = S[P_BLA + 1], bb0 = S[P_BLB], bb1 = S[P_BLB + 1], bc0 = S[P_BLC],
                 bc1 = S[P_BLC + 1], bz0 = S[P_BLZ], bz1 = S[P_BLZ + 1], bz2 = S[P_BLZ + 2];
  uint32_t tw[4];   // omega^(i + k) for this thread's 4 coefficients
  const uint64_t top = a.la > a.lzx ? a.la : a.lzx;
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x * 4;
  for (uint64_t i = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) * 4; i < top; i += stride) {
    // omega^i, i mod 16 (omega^16 = 1 for omega != 0)
    {
      uint32_t x = 1, b = om, e = (uint32_t)(i & 15);
      while (e) { if (e & 1) x = x * b % HFP; b = b * b % HFP; e >>= 1; }
      tw[0] = x;
#pragma unroll
      for (int k = 1; k < 4; k++) tw[k] = tw[k - 1] * om % HFP;
    }
    uint32_t z[6];   // z[k + 2] = Z_H[i + k] mod 17, k = -2 .. 3 (zero outside [0, lz))
    {
      const uint32_t w = load4(a.zh, a.lz, i);
#pragma unroll
      for (int k = 0; k < 4; k++) z[k + 2] = hmod((w >> (8 * k)) & 0xFFu);
      z[0] = (i >= 2 && i - 2 < a.lz) ? a.zh[i - 2] % HFP : 0u;
      z[1] = (i >= 1 && i - 1 < a.lz) ? a.zh[i - 1] % HFP : 0u;
    }
    const uint32_t fa = load4(a.fa, a.n, i), fb = load4(a.fb, a.n, i), fc = load4(a.fc, a.n, i),
                   fz = load4(a.acc, a.n, i), f1 = load4(a.s1, a.n, i), f2 = load4(a.s2, a.n, i),
                   f3 = load4(a.s3, a.n, i);
    uint32_t oA = 0, oB = 0, oC = 0, oZ = 0, oA2 = 0, oB2 = 0, oC2 = 0, oA3 = 0, oB3 = 0, oC3 = 0, oZW = 0, oZ1 = 0;
#pragma unroll
    for (int k = 0; k < 4; k++) {
      const int sh = 8 * k;
      auto byte = [&](uint32_t f) { return (f >> sh) & 0xFFu; };
      const uint32_t c0 = (i + k == 0), c1 = (i + k == 1);
      // (hmod bounds: scalars < 17, bytes < 256: every argument < 16 (16 + 3 * 256 + 256))
      const uint32_t va = hmod(ba0 * z[k + 2] + ba1 * z[k + 1] + byte(fa));
      const uint32_t vb = hmod(bb0 * z[k + 2] + bb1 * z[k + 1] + byte(fb));
      const uint32_t vc = hmod(bc0 * z[k + 2] + bc1 * z[k + 1] + byte(fc));
      const uint32_t vz = hmod(bz0 * z[k + 2] + bz1 * z[k + 1] + bz2 * z[k] + byte(fz));
      oA |= va << sh; oB |= vb << sh; oC |= vc << sh; oZ |= vz << sh;
      oA2 |= hmod((va + c0 * ga + c1 * be) * al) << sh;
      oB2 |= hmod(vb + c0 * ga + c1 * bk1) << sh;
      oC2 |= hmod(vc + c0 * ga + c1 * bk2) << sh;
      oA3 |= hmod((va + be * byte(f1) + c0 * ga) * al) << sh;
      oB3 |= hmod(vb + be * byte(f2) + c0 * ga) << sh;
      oC3 |= hmod(vc + be * byte(f3) + c0 * ga) << sh;
      oZW |= hmod(vz * (om == 0 ? c0 : tw[k])) << sh;
      oZ1 |= hmod((vz + c0 * 16u) * al2) << sh;
    }
    store4(a.cA, a.la, i, oA); store4(a.cB, a.la, i, oB); store4(a.cC, a.la, i, oC);
    // (NULL: not needed by this call -- A2 B2 derived from a_x b_x by t2a_kernel, or a chain whose
    // product comes from another GPU; uniform branches)
    if (a.A2) {
      store4(a.A2, a.la, i, oA2);
      store4(a.B2, a.la, i, oB2);
    }
    if (a.C2) store4(a.C2, a.la, i, oC2);
    if (a.A3) {
      store4(a.A3, a.la, i, oA3); store4(a.B3, a.la, i, oB3); store4(a.C3, a.la, i, oC3);
    }
    store4(a.cZ, a.lzx, i, oZ); store4(a.ZW, a.lzx, i, oZW); store4(a.Z1, a.lzx, i, oZ1);
  }
}

// Round 3's A2 B2 = alpha (a + gamma + beta x)(b + gamma + beta k1 x) (src/plonk.h:409-434) without a
// product of its own: distributing over GF(17),
//   A2 B2 = alpha (ab + gamma (a + b) + beta k1 x a + beta x b + (gamma + beta x)(gamma + beta k1 x)),
// an elementwise pass over a b (round 3's own a_x b_x product) and a, b with a shift of one --
// the same bytes as the 2^(k+1)-point product it replaces (the derived form is exact mod 17).
// 4 coefficients per thread; every pointer 4-byte aligned (prover-internal buffers).
__global__ __launch_bounds__(256) void t2a_kernel(const uint8_t* __restrict__ ab, const uint8_t* __restrict__ a,
                                                  const uint8_t* __restrict__ b, uint64_t la, uint64_t lab,
                                                  const uint8_t* __restrict__ S, uint8_t* __restrict__ out) {
  const uint32_t al = S[S_ALPHA], be = S[S_BETA], ga = S[S_GAMMA], bk1 = S[S_BK1];
  const uint32_t K[3] = {ga * ga, ga * (bk1 + be), be * bk1};   // (gamma + beta x)(gamma + beta k1 x)
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x * 4;
  for (uint64_t i = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) * 4; i < lab; i += stride) {
    const uint32_t wab = load4(ab, lab, i);
    uint32_t wa = 0, wb = 0, pa = 0, pb = 0;   // a[i..i+3], b[i..i+3], a[i-1], b[i-1]
    if (i <= la) {                             // (a, b and their shifts vanish past index la)
      wa = load4(a, la, i);
      wb = load4(b, la, i);
      if (i) {
        pa = load4(a, la, i - 4) >> 24;
        pb = load4(b, la, i - 4) >> 24;
      }
    }
    uint32_t o = 0;
#pragma unroll
    for (int k = 0; k < 4; k++) {
      const int sh = 8 * k;
      const uint32_t ak = (wa >> sh) & 0xFFu, bk = (wb >> sh) & 0xFFu;
      const uint32_t am = k ? (wa >> (sh - 8)) & 0xFFu : pa, bm = k ? (wb >> (sh - 8)) & 0xFFu : pb;
      const uint64_t j = i + k;
      // (hmod bound: 16 + 16 * 32 + 2 * 16 * 16 + 289 < 69632)
      const uint32_t v = ((wab >> sh) & 0xFFu) + ga * (ak + bk) + bk1 * am + be * bm + (j < 3 ? K[j] : 0u);
      o |= hmod(hmod(v) * al) << sh;
    }
    store4(out, lab, i, o);
  }
}

// several independent lincombs in one launch (blockIdx.y = which), all 16-byte aligned
constexpr int LCB_MAX = 8;
struct LcBatch {
  LcArgs a[LCB_MAX];
};
__global__ __launch_bounds__(256) void lincomb16_batch_kernel(LcBatch b, const uint8_t* __restrict__ S) {
  const LcArgs& a = b.a[blockIdx.y];
  uint32_t cf[LC_MAX];
#pragma unroll
  for (int t = 0; t < LC_MAX; t++) cf[t] = t < a.nt ? S[a.slot[t]] : 0u;
  const uint32_t sc = S[a.scale];
  const uint32_t c0 = a.c0 >= 0 ? S[a.c0] : 0u, c1 = a.c1 >= 0 ? S[a.c1] : 0u;
  const uint32_t x = a.twist >= 0 ? S[a.twist] : 1u;
  uint32_t tw[16];
  tw[0] = 1;
#pragma unroll
  for (int k = 1; k < 16; k++) tw[k] = tw[k - 1] * x % HFP;
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x * 16;
  for (uint64_t i = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) * 16; i < a.out_len; i += stride) {
    uint32_t acc[16];
#pragma unroll
    for (int k = 0; k < 16; k++) acc[k] = 0;
    if (i == 0) { acc[0] = c0; acc[1] = c1; }
#pragma unroll
    for (int t = 0; t < LC_MAX; t++) {
      if (t < a.nt && i < a.len[t]) {
        uint32_t w[4];
        load16(a.p[t], a.len[t], i, w);
#pragma unroll
        for (int k = 0; k < 16; k++) acc[k] += cf[t] * ((w[k >> 2] >> (8 * (k & 3))) & 0xFFu);
      }
    }
    uint32_t o[4] = {0, 0, 0, 0};
#pragma unroll
    for (int k = 0; k < 16; k++) {
      uint32_t v = hmod(hmod(acc[k]) * sc);   // (acc <= 16 terms x 16 x 255 + 32 < 69632)
      if (a.twist >= 0) v = hmod(v * (x == 0 ? (i + k == 0 ? 1u : 0u) : tw[k]));
      o[k >> 2] |= v << (8 * (k & 3));
    }
    if (i + 16 <= a.out_len) {
      *reinterpret_cast<uint4*>(a.out + i) = make_uint4(o[0], o[1], o[2], o[3]);
    } else {
#pragma unroll
      for (int k = 0; k < 16; k++)
        if (i + k < a.out_len) a.out[i + k] = (uint8_t)(o[k >> 2] >> (8 * (k & 3)));
    }
  }
}

// three slices of t(x) into the commitment arena in one launch (poly_slice, src/plonk.h:513-519)
struct Copy3 {
  const uint8_t* src[3];
  uint8_t* dst[3];
  uint64_t len[3];
};
__global__ __launch_bounds__(256) void copy3_kernel(Copy3 c) {
  const int s = blockIdx.y;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < c.len[s]; i += (uint64_t)gridDim.x * blockDim.x)
    c.dst[s][i] = c.src[s][i];
}

// ------------------------------------------------------------------ poly_eval (batched)
// Horner of src/poly.h:265-272 == sum c_i x^i mod 17; x^i = x^(i mod 16) for x != 0.
constexpr int EV_MAX = 16;   // evaluations per launch (arrival words)
constexpr int EV_ROWS = 24;  // grid rows: a long evaluation runs as several rows (EvArgs::grp)
#ifndef PLK_SLICE_WORDS
#define PLK_SLICE_WORDS 1   // numdiv_kernel: t_lo / t_mid / t_hi stored a word (or two halves) at a time
#endif
#ifndef PLK_EV_SPLIT
#define PLK_EV_SPLIT 1   // long evaluations as several grid rows (make_evargs)
#endif
#ifndef PLK_CP_BX
#define PLK_CP_BX 227   // commit_pack_kernel: blocks per MSM row at most (2048 / 9)
#endif
#ifndef PLK_MSM_ROW_LENS
#define PLK_MSM_ROW_LENS 1   // commitment MSMs over each row's own length (0: the arena stride's cmax)
#endif
#ifndef PLK_EV_BLOCKS
#define PLK_EV_BLOCKS 64
#endif
constexpr int EV_BLOCKS = PLK_EV_BLOCKS;   // x 256 threads x 4 uint4 loads in flight each
constexpr int TICK_STRIDE = 32;   // one 128-byte line per arrival word
constexpr int AGG_CHUNK = 4096;   // round 5's scan chunk (SCAN_B) as aggregated by the evaluation rows
enum EvPost : int { EV_POST_NONE = 0, EV_POST_ACC = 1, EV_POST_R4 = 4 };
struct EvArgs {
  const uint8_t* p[EV_ROWS];
  uint64_t len[EV_ROWS];
  int xslot[EV_ROWS];
  int out[EV_ROWS];
  int vec[EV_ROWS];   // pointer 16-byte aligned: uint4 loads
  // row -> evaluation: a row is coefficients [off, off + len) of its evaluation's polynomial
  // (off = 0 mod 16, so x^(off + i) = x^i); the evaluation's parts rows share its arrival word
  int grp[EV_ROWS];
  int parts[EV_ROWS];
  int first[EV_ROWS];   // off == 0 (the row that holds p[0])
  // the row's partial enters its evaluation times x^mexp (a slice of a longer polynomial whose offset
  // is not 0 mod 16: t(x) from t_lo / t_mid / t_hi)
  int mexp[EV_ROWS];
  // chunk aggregates for round 5's divisions (PLK_OPT_PROVE_EVAL_AGG): col >= 0 stores, for every
  // 4096-coefficient chunk c of the row's polynomial, sum_{i in c} p[i] x^i mod 17 at
  // agg[16 (coff + c) + col] (coff: the row's first chunk, a split row's offset / 4096)
  int col[EV_ROWS];
  int coff[EV_ROWS];
  uint8_t* agg;
  int ne;               // evaluations (the top ticket counts them)
  int nr;               // rows
  int post;             // scalar program the last block runs (EvPost)
};

__device__ void scalars_r45(uint8_t* S, uint32_t tz);

// Block bx of BX of evaluation e (eval_kernel's rows, or extra blocks of another launch): its
// partial with a ticket to the row's arrival word; the row's last block writes S[out] and, with
// `top`, takes a ticket on the top word -- whose last taker runs the round's scalar program.
__device__ __forceinline__ void eval_row_block(const EvArgs& a, int e, uint32_t bx, uint32_t BX, uint8_t* S,
                                               uint32_t* tick, uint32_t* stat, bool top) {
  const uint32_t x = S[a.xslot[e]];
  uint32_t pw[16];
  pw[0] = 1;
#pragma unroll
  for (int j = 1; j < 16; j++) pw[j] = pw[j - 1] * x % HFP;
  const uint8_t* p = a.p[e];
  const uint64_t n = a.len[e];
  uint32_t acc = 0;
  const uint64_t gid = (uint64_t)bx * blockDim.x + threadIdx.x;
  const uint64_t stride = (uint64_t)BX * blockDim.x * 16;
  if (x == 0) {                       // poly_eval(p, 0) = p[0]
    if (gid == 0 && n && a.first[e]) acc = p[0];
  } else if (a.col[e] >= 0) {
    // a wave per 4096-coefficient chunk (4 x 1 KiB loads in flight per lane), so the chunk's sum is
    // one wave reduction: it is stored as round 5's scan aggregate and added into the evaluation.
    // (make_evargs: such rows are readable in whole 16-byte chunks, split at multiples of 4096)
    const uint32_t lane = threadIdx.x & 63u, wv = threadIdx.x >> 6;
    const uint64_t nch = (n + AGG_CHUNK - 1) / AGG_CHUNK;
    for (uint64_t c = (uint64_t)bx * (blockDim.x >> 6) + wv; c < nch; c += (uint64_t)BX * (blockDim.x >> 6)) {
      uint32_t w[4][4];
#pragma unroll
      for (int u = 0; u < 4; u++) load16_masked(p, n, c * AGG_CHUNK + u * 1024 + lane * 16, w[u]);
      uint32_t s = 0;
#pragma unroll
      for (int u = 0; u < 4; u++)
#pragma unroll
        for (int k = 0; k < 16; k++) s += pw[k] * ((w[u][k >> 2] >> (8 * (k & 3))) & 0xFFu);   // (<= 64 x 16 x 255)
      s %= HFP;
#pragma unroll
      for (int d = 32; d > 0; d >>= 1) s += __shfl_xor(s, d, 64);   // (<= 64 x 16)
      if (lane == 0) {
        s = hmod(s);
        a.agg[16 * ((uint64_t)a.coff[e] + c) + a.col[e]] = (uint8_t)s;
        acc += s;
      }
    }
    acc = hmod(acc);
  } else if (a.vec[e] == 2) {         // readable in whole chunks: 4 loads in flight per thread
    for (uint64_t i0 = gid * 16; i0 < n; i0 += 4 * stride) {
      uint32_t w[4][4];
#pragma unroll
      for (int u = 0; u < 4; u++) load16_masked(p, n, i0 + u * stride, w[u]);
#pragma unroll
      for (int u = 0; u < 4; u++) {
        uint32_t s = 0;
#pragma unroll
        for (int k = 0; k < 16; k++) s += pw[k] * ((w[u][k >> 2] >> (8 * (k & 3))) & 0xFFu);
        acc = (acc + s) % HFP;
      }
    }
  } else if (a.vec[e]) {              // 16 coefficients per step: i = 0 mod 16 so x^(i+k) = x^k
    for (uint64_t i = gid * 16; i < n; i += stride) {
      uint32_t w[4];
      load16(p, n, i, w);
      uint32_t s = 0;
#pragma unroll
      for (int k = 0; k < 16; k++) s += pw[k] * ((w[k >> 2] >> (8 * (k & 3))) & 0xFFu);
      acc = (acc + s) % HFP;
    }
  } else {
    for (uint64_t i = gid * 16; i < n; i += stride) {
      uint32_t s = 0;
#pragma unroll
      for (int k = 0; k < 16; k++) s += i + k < n ? pw[k] * p[i + k] : 0u;
      acc = (acc + s) % HFP;
    }
  }
  // block sum: wave shuffles, then one barrier (acc < 17: the sum fits easily)
#pragma unroll
  for (int d = 32; d > 0; d >>= 1) acc += __shfl_xor(acc, d, 64);
  __shared__ uint32_t red[4];
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = acc;
  __syncthreads();
  if (threadIdx.x != 0) return;
  // the partial travels inside the atomic (no fence: a device-scope release per block costs an
  // L2 writeback each, 2048 of them took 60 us): row word = sum | arrivals << 32
  const uint32_t mine = (red[0] + red[1] + red[2] + red[3]) % HFP * pw[a.mexp[e]] % HFP;
  unsigned long long* row = reinterpret_cast<unsigned long long*>(tick) + a.grp[e] * (TICK_STRIDE / 2);
  const unsigned long long old = atomicAdd(row, (unsigned long long)mine | (1ull << 32));
  if ((uint32_t)(old >> 32) != BX * (uint32_t)a.parts[e] - 1) return;
  *row = 0;                                               // re-armed for the next launch
  // the row's last block publishes the value: only these <= EV_MAX blocks fence
  S[a.out[e]] = (uint8_t)(((uint32_t)old + mine) % HFP);
  __threadfence();
  if (!top) return;
  uint32_t* topw = tick + EV_MAX * TICK_STRIDE;
  if (atomicAdd(topw, 1u) != (uint32_t)a.ne - 1) return;
  __threadfence();
  *topw = 0;
  if (a.post == EV_POST_R4) scalars_r45(S, S[S_TZ]);   // round 4's scalars (incl. r_z) and round 5's (w_z constant)
  if (a.post == EV_POST_ACC) stat[ST_ACC] = S[S_ACCW];   // acc_x(omega^n), src/plonk.h:366-368
}

// One launch per batch of evaluations: blockIdx.y = evaluation, EV_BLOCKS blocks each.  Every
// block adds its partial sum with a ticket to its evaluation's arrival word; the last block of
// an evaluation adds the finished value with a ticket to the top word; the last of those writes
// every S[out] and runs the round's scalar program -- the partial / final / scalar kernels of a
// three-launch chain in one.
// (optional) commitments that do not wait for round 5, run as extra grid rows of an earlier launch
// (round 5's scan, or round 4's evaluations): rows y >= nd are log-form MSMs of arena rows
// 0 .. nrows - 1 on X blocks each
// points per commitment row: each row's own upper-bound length (the arena row is zero past it),
// not the arena's stride -- w_z(x)'s quotient is ~2n long, the other eight ~n
struct MsmRowLens {
  uint64_t n[9];
};
struct EarlyMsm {
  const uint8_t* logs;
  const uint8_t* arena;
  uint64_t cstride;
  MsmRowLens rl;
  PlkMsmResult* res;
  const uint32_t* exp_words;
  int nrows, nd;
  uint32_t X;
};
__global__ __launch_bounds__(256) void eval_kernel(EvArgs a, uint8_t* __restrict__ S, uint32_t* __restrict__ tick,
                                                   uint32_t* __restrict__ stat, EarlyMsm em) {
  if ((int)blockIdx.y >= a.nr) {   // (uniform) an early commitment row
    __shared__ uint32_t etab[PLK_GROUP_ORDER];
    __shared__ uint32_t wsum[256 / PLK_WAVE];
    __shared__ uint32_t wbad[256 / PLK_WAVE];
    const int r = (int)blockIdx.y - a.nr;
    (void)msm_log_block<256>(em.logs, em.arena + (uint64_t)r * em.cstride, em.rl.n[r], blockIdx.x, gridDim.x, (uint32_t)r,
                             em.res + r, em.exp_words, etab, wsum, wbad);
    return;
  }
  eval_row_block(a, (int)blockIdx.y, blockIdx.x, gridDim.x, S, tick, stat, true);
}

// ------------------------------------------------------------------ poly_divide
// (a) divisor L x^m + c (Z_H of a multiplicative subgroup is x^n - 1): the long division
// of src/poly.h:124-177 gives q[j] = L^-1 (num[j+m] - c q[j+m]) and rem[r] = num[r] - c q[r]
// (r < m) -- independent chains per residue r mod m, walked top-down by one thread each.
__global__ __launch_bounds__(256) void divide_binomial_kernel(const uint8_t* __restrict__ num, uint64_t nl,
                                                              uint64_t m, uint32_t lead, uint32_t c,
                                                              uint8_t* __restrict__ q, uint64_t ql,
                                                              uint32_t* __restrict__ rem_flag) {
  const uint64_t r0 = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const uint64_t r = r0 < m ? r0 : m;   // lanes past m idle but stay for the wave vote
  const uint32_t li = hinv(lead);
  const uint32_t nc = hneg(c);
  uint32_t prev = 0;   // q[j + m]
  const uint64_t cnt = (r < m && nl > m && r < ql) ? (ql - 1 - r) / m + 1 : 0;   // chain length
  if (cnt <= 8) {
    // the prover's chains are ~4 long: issue every load of the chain first, then walk it
    // (a load per step inside the loop serialised one memory latency per step)
    uint32_t w[8];
#pragma unroll
    for (int t = 0; t < 8; t++) w[t] = (uint64_t)t < cnt ? num[r + (cnt - 1 - t) * m + m] : 0u;
#pragma unroll
    for (int t = 0; t < 8; t++) {
      if ((uint64_t)t < cnt) {
        const uint32_t v = (w[t] + nc * prev) % HFP * li % HFP;
        q[r + (cnt - 1 - t) * m] = (uint8_t)v;
        prev = v;
      }
    }
  } else {
    uint64_t j = r + (cnt - 1) * m;   // top of the chain
    for (;;) {
      const uint32_t v = (num[j + m] + nc * prev) % HFP * li % HFP;
      q[j] = (uint8_t)v;
      prev = v;
      if (j < m) break;
      j -= m;
    }
  }
  const uint32_t rv = (r < m && r < nl) ? (num[r] + nc * prev) % HFP : 0u;   // prev = q[r] (0 if none)
  // one flag word for the whole grid: vote per block, and skip the atomic once it is set
  // (same-address atomics from every wave serialise in one L2 channel)
  if (__syncthreads_or(rv != 0) && threadIdx.x == 0 && __hip_atomic_load(rem_flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0)
    atomicOr(rem_flag, 1u);
}

// The same with 4 consecutive residues per thread (m % 4 == 0, num / q 4-byte aligned): one
// dword per chain element, loaded before the chains are walked.  Lanes of a residue whose chain
// is one shorter than its word's first residue skip the word's top element (and do not store it).
// cq, cr: ql - 1 = cq m + cr (host-side), so a chain has cq + 1 elements for r <= cr and cq
// after (no 64-bit division on the device: a software routine of ~100 instructions per call)
__global__ __launch_bounds__(256) void divide_binomial4_kernel(const uint8_t* __restrict__ num, uint64_t nl,
                                                               uint64_t m, uint32_t lead, uint32_t c,
                                                               uint8_t* __restrict__ q, uint64_t ql, uint64_t cq,
                                                               uint64_t cr, uint8_t* __restrict__ rem_part) {
  const uint64_t r0 = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) * 4;
  const uint32_t li = hinv(lead);
  const uint32_t nc = hneg(c);
  auto chain = [&](uint64_t r) -> uint64_t { return (r < m && nl > m && r < ql) ? (r <= cr ? cq + 1 : cq) : 0; };
  const uint64_t cnt0 = chain(r0);   // the longest of the 4 (chain length falls with r)
  uint32_t rv = 0;
  if (cnt0 <= 8) {
    uint32_t w[8];
#pragma unroll
    for (int k = 0; k < 8; k++)
      w[k] = (uint64_t)k < cnt0 ? *reinterpret_cast<const uint32_t*>(num + r0 + (cnt0 - 1 - k) * m + m) : 0u;
    uint32_t prev[4] = {0, 0, 0, 0}, skip[4];
#pragma unroll
    for (int b = 0; b < 4; b++) skip[b] = (uint32_t)(cnt0 - chain(r0 + b));   // 0 or 1 (or cnt0 past the end)
#pragma unroll
    for (int k = 0; k < 8; k++) {
      if ((uint64_t)k < cnt0) {
        uint32_t o = 0;
#pragma unroll
        for (int b = 0; b < 4; b++) {
          if ((uint32_t)k >= skip[b]) {
            const uint32_t v = hmod((((w[k] >> (8 * b)) & 0xFFu) + nc * prev[b]) * li);   // (<= (255 + 256) x 16)
            prev[b] = v;
            o |= v << (8 * b);
          }
        }
        uint8_t* dst = q + r0 + (cnt0 - 1 - k) * m;
        if (skip[0] == 0 && skip[3] == 0) *reinterpret_cast<uint32_t*>(dst) = o;
        else
#pragma unroll
          for (int b = 0; b < 4; b++)
            if ((uint32_t)k >= skip[b]) dst[b] = (uint8_t)(o >> (8 * b));
      }
    }
#pragma unroll
    for (int b = 0; b < 4; b++) {
      const uint64_t r = r0 + b;
      if (r < m && r < nl && (num[r] + nc * prev[b]) % HFP) rv = 1;   // prev = q[r] (0 if none)
    }
  } else {
    for (int b = 0; b < 4; b++) {
      const uint64_t r = r0 + b;
      const uint64_t cnt = chain(r);
      uint32_t prev = 0;
      for (uint64_t t = 0; t < cnt; t++) {
        const uint64_t j = r + (cnt - 1 - t) * m;
        const uint32_t v = (num[j + m] + nc * prev) % HFP * li % HFP;
        q[j] = (uint8_t)v;
        prev = v;
      }
      if (r < m && r < nl && (num[r] + nc * prev) % HFP) rv = 1;
    }
  }
  // one vote byte per block (trim_pack_kernel ORs them into the status word): the blocks run
  // together, so a "skip if already set" atomic would still serialise ~1000 same-address ORs
  const int vote = __syncthreads_or(rv != 0);
  if (threadIdx.x == 0) rem_part[blockIdx.x] = vote ? 1 : 0;
}

// A word's bytes 0 / 2 (lanes02) or 1 / 3 (lanes13) as two 16-bit lanes for the two-bytes-per-
// multiply lincombs.  The empty asm hides the mask from the optimizer: this compiler (ROCm 7.2
// clang 22, gfx942 / gfx950) rewrites a straight-line sum of byte x (w & 0x00FF00FF) products as
// one v_dot4_u32_u8 over byte 0 alone, dropping the byte-2 lane (tools/swar_dot4_repro.hip).
__device__ __forceinline__ uint32_t lanes02(uint32_t w) {
  uint32_t m = w & 0x00FF00FFu;
  asm("" : "+v"(m));
  return m;
}
__device__ __forceinline__ uint32_t lanes13(uint32_t w) {
  uint32_t m = (w >> 8) & 0x00FF00FFu;
  asm("" : "+v"(m));
  return m;
}

// t(x) in one launch: the numerator lincomb (src/plonk.h:494-503) evaluated per chain element
// (no numerator buffer: its dwords come straight from the 8 product / q_c terms), the Z_H
// division of divide_binomial4_kernel, and the t_lo / t_mid / t_hi slices (src/plonk.h:513-519)
// written into the commitment arena next to t(x) itself.
struct Slices3 {
  uint8_t* dst[3];
  uint64_t len[3];
  uint64_t part;
};
// NT terms, branch-free: every load is issued (a position past a term's length reads the term's
// first dword and is masked), so the chain's loads go out together -- loads under divergent
// branches each waited for vmcnt(0).  Terms are 4-byte aligned and readable up to their length
// rounded up to 4 (checked on the host).
template <int NT>
__device__ __forceinline__ uint32_t lc_word(const LcArgs& a, const uint32_t (&cf)[LC_MAX], uint32_t sc, uint32_t c0,
                                            uint32_t c1, uint64_t x) {   // x = 0 mod 4
  uint32_t acc[4] = {x == 0 ? c0 : 0u, x == 0 ? c1 : 0u, 0u, 0u};
#pragma unroll
  for (int t = 0; t < NT; t++) {
    const uint64_t len = a.len[t];
    const bool in = x < len;
    const uint32_t wv = *reinterpret_cast<const uint32_t*>(a.p[t] + (in ? x : 0));
    const uint32_t mask = x + 4 <= len ? 0xFFFFFFFFu : (in ? (1u << (8 * (uint32_t)(len - x))) - 1u : 0u);
    const uint32_t w = wv & mask;
#pragma unroll
    for (int b = 0; b < 4; b++) acc[b] += cf[t] * ((w >> (8 * b)) & 0xFFu);
  }
  uint32_t o = 0;
#pragma unroll
  for (int b = 0; b < 4; b++) o |= hmod(hmod(acc[b]) * sc) << (8 * b);   // (acc <= 8 x 16 x 255 + 16)
  return o;
}
template <int NT, int KMAX>
__global__ __launch_bounds__(256) void numdiv_kernel(LcArgs a, const uint8_t* __restrict__ S, uint64_t m, uint32_t lead,
                                                     uint32_t c, uint8_t* __restrict__ q, uint64_t ql, uint64_t cq,
                                                     uint64_t cr, Slices3 sl, uint8_t* __restrict__ rem_part) {
  uint32_t cf[LC_MAX];
#pragma unroll
  for (int t = 0; t < LC_MAX; t++) cf[t] = t < NT ? S[a.slot[t]] : 0u;
  const uint32_t sc = S[a.scale];
  const uint32_t c0 = a.c0 >= 0 ? S[a.c0] : 0u, c1 = a.c1 >= 0 ? S[a.c1] : 0u;
  const uint64_t nl = a.out_len;
  const uint64_t r0 = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) * 4;
  const uint32_t li = hinv(lead);
  const uint32_t nc = hneg(c);
  auto chain = [&](uint64_t r) -> uint64_t { return (r < m && nl > m && r < ql) ? (r <= cr ? cq + 1 : cq) : 0; };
  const uint64_t cnt0 = chain(r0);
  uint32_t w[KMAX];   // chains are at most KMAX = cq + 1 long (host): no branch around the loads
#pragma unroll
  for (int k = 0; k < KMAX; k++) {
    const uint64_t x = (uint64_t)k < cnt0 ? r0 + (cnt0 - 1 - k) * m + m : 0;   // shorter chains: drop
    const uint32_t v = lc_word<NT>(a, cf, sc, c0, c1, x);
    w[k] = (uint64_t)k < cnt0 ? v : 0u;
  }
  const uint32_t wr = lc_word<NT>(a, cf, sc, c0, c1, r0 < m ? r0 : 0);   // num[r0 .. r0+3] (remainders)
  uint32_t prev[4] = {0, 0, 0, 0}, skip[4];
#pragma unroll
  for (int b = 0; b < 4; b++) skip[b] = (uint32_t)(cnt0 - chain(r0 + b));
#pragma unroll
  for (int k = 0; k < KMAX; k++) {
    if ((uint64_t)k < cnt0) {
      uint32_t o = 0;
#pragma unroll
      for (int b = 0; b < 4; b++) {
        if ((uint32_t)k >= skip[b]) {
          const uint32_t v = hmod((((w[k] >> (8 * b)) & 0xFFu) + nc * prev[b]) * li);   // (<= (255 + 256) x 16)
          prev[b] = v;
          o |= v << (8 * b);
        }
      }
      const uint64_t j0 = r0 + (cnt0 - 1 - k) * m;
      if (skip[0] == 0 && skip[3] == 0) *reinterpret_cast<uint32_t*>(q + j0) = o;
      else
#pragma unroll
        for (int b = 0; b < 4; b++)
          if ((uint32_t)k >= skip[b]) q[j0 + b] = (uint8_t)(o >> (8 * b));
      // the slices: a whole word inside one slice as one dword (or two 16-bit halves: t_mid
      // starts at n + 2 = 2 mod 4), else byte by byte
      const int s0 = j0 < sl.part ? 0 : (j0 < 2 * sl.part ? 1 : 2);
      const uint64_t o0 = j0 - (uint64_t)s0 * sl.part;
      uint8_t* const d0 = sl.dst[s0] + o0;
      if (PLK_SLICE_WORDS && skip[0] == 0 && skip[3] == 0 && o0 + 4 <= sl.len[s0] &&
          (s0 == 2 || o0 + 4 <= sl.part) && ((uintptr_t)d0 & 1) == 0) {
        if (((uintptr_t)d0 & 3) == 0) {
          *reinterpret_cast<uint32_t*>(d0) = o;
        } else {
          reinterpret_cast<uint16_t*>(d0)[0] = (uint16_t)o;
          reinterpret_cast<uint16_t*>(d0)[1] = (uint16_t)(o >> 16);
        }
      } else {
#pragma unroll
        for (int b = 0; b < 4; b++) {
          if ((uint32_t)k < skip[b]) continue;
          const uint64_t j = j0 + b;
          const int si = j < sl.part ? 0 : (j < 2 * sl.part ? 1 : 2);
          const uint64_t off = j - (uint64_t)si * sl.part;
          if (off < sl.len[si]) sl.dst[si][off] = (uint8_t)(o >> (8 * b));
        }
      }
    }
  }
  uint32_t rv = 0;
#pragma unroll
  for (int b = 0; b < 4; b++) {
    const uint64_t r = r0 + b;
    if (r < m && r < nl && hmod(((wr >> (8 * b)) & 0xFFu) + nc * prev[b])) rv = 1;
  }
  const int vote = __syncthreads_or(rv != 0);
  if (threadIdx.x == 0) rem_part[blockIdx.x] = vote ? 1 : 0;
}

// (b) divisor d1 x + d0: the long division gives q[j] = b num[j+1] + a q[j+1] with
// a = -d0/d1, b = 1/d1, i.e. q[j] = b a^-(j+1) sum_{i>j} num[i] a^i  (a != 0; a^i = a^(i mod 16)).
// The prover only divides by x - z and x - z omega (d1 = 1).  Two-phase suffix scan over
// 4096-element blocks: block aggregates, then each block reduces the aggregates after it itself.
constexpr int SCAN_T = 256, SCAN_E = 16, SCAN_B = SCAN_T * SCAN_E;
static_assert(SCAN_B == AGG_CHUNK, "the evaluation rows' chunk aggregates are the scan's");
// Round 5's two divisions (by x - z and by x - z omega) are independent: one launch per phase
// for both (blockIdx.y / the carry block = the division).
struct LinDiv {
  const uint8_t* num;
  uint64_t nl;
  int aslot;
  int nb;              // scan blocks
  uint8_t* q;
  uint32_t* flag;
  uint32_t* bsum;
  int vec;             // num and q 16-byte aligned: uint4 loads / stores
};

// wave-level (64 lanes) sums by cross-lane shuffles: no LDS, no barrier
__device__ __forceinline__ uint32_t wave_sum(uint32_t x) {
#pragma unroll
  for (int d = 32; d > 0; d >>= 1) x += __shfl_xor(x, d, 64);
  return x;
}
// inclusive suffix sum: lane l gets the sum over lanes l .. 63
__device__ __forceinline__ uint32_t wave_suffix(uint32_t x) {
  const int lane = (int)(threadIdx.x & 63);
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const uint32_t v = __shfl_down(x, d, 64);
    if (lane + d < 64) x += v;
  }
  return x;
}
// block sum of SCAN_T threads' values (< 2^26 / SCAN_T each) for thread 0: wave sums + one barrier
__device__ __forceinline__ uint32_t scan_block_sum(uint32_t x) {
  __shared__ uint32_t ws[SCAN_T / 64];
  x = wave_sum(x);
  if ((threadIdx.x & 63) == 0) ws[threadIdx.x >> 6] = x;
  __syncthreads();
  uint32_t t = 0;
#pragma unroll
  for (int u = 0; u < SCAN_T / 64; u++) t += ws[u];
  return t;
}
struct LinDivs {
  LinDiv d[2];
};

// acc[k] = c0 [k == 0] + c1 [k == 1] + sum_t cf[t] p_t[i + k], k < 16 (i = 0 mod 16; terms read in
// whole 16-byte chunks, masked past their lengths).  The products go two bytes at a time: a word's
// bytes 0 / 2 and 1 / 3 as two 16-bit lanes (w & 0x00FF00FF, (w >> 8) & 0x00FF00FF) times cf[t] by
// one 24-bit multiply each -- 16 x 16 x 255 + 32 < 2^16, so no lane carries into the next -- half
// the multiplies and extracts of a per-byte loop.
// p readable in whole 4 NW-byte chunks up to len (aligned to them): one unconditional load at a
// clamped address, bytes past len masked (load16_masked for NW = 4)
template <int NW>
__device__ __forceinline__ void loadw_masked(const uint8_t* p, uint64_t len, uint64_t i, uint32_t (&w)[NW]) {
  const bool in = i < len;
  uint32_t v[NW];
  if constexpr (NW == 4) {
    const uint4 q = *reinterpret_cast<const uint4*>(p + (in ? i : 0));
    v[0] = q.x; v[1] = q.y; v[2] = q.z; v[3] = q.w;
  } else {
    static_assert(NW == 2, "8 or 16 bytes");
    const uint2 q = *reinterpret_cast<const uint2*>(p + (in ? i : 0));
    v[0] = q.x; v[1] = q.y;
  }
#pragma unroll
  for (int k = 0; k < NW; k++) {
    const int64_t cnt = in ? (int64_t)len - (int64_t)(i + 4 * k) : 0;   // valid bytes in word k
    w[k] = cnt >= 4 ? v[k] : (cnt <= 0 ? 0u : v[k] & ((1u << (8 * cnt)) - 1u));
  }
}
template <int NW>
__device__ __forceinline__ void lc_swar(const LcArgs& a, const uint32_t (&cf)[LC_MAX], uint32_t c0, uint32_t c1,
                                        uint64_t i, uint32_t (&acc)[4 * NW]) {
  uint32_t E[NW] = {}, O[NW] = {};   // even / odd bytes
  E[0] = i == 0 ? c0 : 0u;
  O[0] = i == 0 ? c1 : 0u;
#pragma unroll
  for (int t = 0; t < LC_MAX; t++) {
    if (t < a.nt) {   // uniform
      uint32_t w[NW];
      loadw_masked<NW>(a.p[t], a.len[t], i, w);
#pragma unroll
      for (int q = 0; q < NW; q++) {
        E[q] += __umul24(cf[t], lanes02(w[q]));
        O[q] += __umul24(cf[t], lanes13(w[q]));
      }
    }
  }
#pragma unroll
  for (int q = 0; q < NW; q++) {
    acc[4 * q] = E[q] & 0xFFFFu;
    acc[4 * q + 1] = O[q] & 0xFFFFu;
    acc[4 * q + 2] = E[q] >> 16;
    acc[4 * q + 3] = O[q] >> 16;
  }
}
__device__ __forceinline__ void lc16_swar(const LcArgs& a, const uint32_t (&cf)[LC_MAX], uint32_t c0, uint32_t c1,
                                          uint64_t i, uint32_t (&acc)[16]) {
  lc_swar<4>(a, cf, c0, c1, i, acc);
}

__global__ __launch_bounds__(SCAN_T) void lin_scan_sums_kernel(LinDivs L, const uint8_t* __restrict__ S) {
  const LinDiv& D = L.d[blockIdx.y];
  if ((int)blockIdx.x >= D.nb) return;
  const uint8_t* num = D.num;
  const uint64_t nl = D.nl;
  const uint32_t a = S[D.aslot];
  uint32_t pw[16];
  pw[0] = 1;
#pragma unroll
  for (int j = 1; j < 16; j++) pw[j] = pw[j - 1] * a % HFP;
  const uint64_t base = (uint64_t)blockIdx.x * SCAN_B + threadIdx.x;
  uint32_t acc = 0;
#pragma unroll
  for (int k = 0; k < SCAN_E; k++) {
    const uint64_t i = base + (uint64_t)k * SCAN_T;
    if (i < nl && i > 0) acc += num[i] * pw[i & 15];
  }
  const uint32_t t = scan_block_sum(acc % HFP);
  if (threadIdx.x == 0) D.bsum[blockIdx.x] = t % HFP;
}

// Round 5's two numerators (w_z(x)'s lincomb, z(x) - z_omega_z) and the scan's block aggregates
// in one launch: block (c, d) writes numerator d's coefficients [4096 c, 4096 (c+1)) and their
// aggregate sum_{i > 0} num[i] a^i.  Every term is 16-byte aligned and readable in whole 16-byte
// chunks up to its length (host-checked), so each term's uint4 load is issued unconditionally
// (clamped address, masked bytes) and all of them are in flight together.
__global__ __launch_bounds__(SCAN_T) void lincomb_scan_kernel(LcBatch b, LinDivs L, const uint8_t* __restrict__ S,
                                                             EarlyMsm em) {
  if ((int)blockIdx.y >= em.nd) {   // (uniform) an early commitment row
    __shared__ uint32_t etab[PLK_GROUP_ORDER];
    __shared__ uint32_t wsum[SCAN_T / PLK_WAVE];
    __shared__ uint32_t wbad[SCAN_T / PLK_WAVE];
    const int r = (int)blockIdx.y - em.nd;
    if (blockIdx.x >= em.X) return;
    (void)msm_log_block<SCAN_T>(em.logs, em.arena + (uint64_t)r * em.cstride, em.rl.n[r], blockIdx.x, em.X, (uint32_t)r,
                                em.res + r, em.exp_words, etab, wsum, wbad);
    return;
  }
  const int d = blockIdx.y;
  const LcArgs& a = b.a[d];
  const LinDiv& D = L.d[d];
  if ((int)blockIdx.x >= D.nb) return;
  uint32_t cf[LC_MAX];
#pragma unroll
  for (int t = 0; t < LC_MAX; t++) cf[t] = t < a.nt ? S[a.slot[t]] : 0u;
  const uint32_t sc = S[a.scale];
  const uint32_t c0 = a.c0 >= 0 ? S[a.c0] : 0u, c1 = a.c1 >= 0 ? S[a.c1] : 0u;
  const uint64_t i = (uint64_t)blockIdx.x * SCAN_B + (uint64_t)threadIdx.x * SCAN_E;
  uint32_t acc[16];
  lc16_swar(a, cf, c0, c1, i, acc);
  const uint32_t av = S[D.aslot];
  uint32_t pw[16];
  pw[0] = 1;
#pragma unroll
  for (int j = 1; j < 16; j++) pw[j] = pw[j - 1] * av % HFP;
  uint32_t o[4] = {0, 0, 0, 0}, agg = 0;
#pragma unroll
  for (int k = 0; k < 16; k++) {
    const uint32_t v = i + k < a.out_len ? hmod(hmod(acc[k]) * sc) : 0u;   // (acc <= 16 x 16 x 255 + 32)
    o[k >> 2] |= v << (8 * (k & 3));
    if (i + k > 0) agg += v * pw[k];   // (i + k) mod 16 = k
  }
  if (i + 16 <= a.out_len) {
    *reinterpret_cast<uint4*>(a.out + i) = make_uint4(o[0], o[1], o[2], o[3]);
  } else {
#pragma unroll
    for (int k = 0; k < 16; k++)
      if (i + k < a.out_len) a.out[i + k] = (uint8_t)(o[k >> 2] >> (8 * (k & 3)));
  }
  const uint32_t t = scan_block_sum(agg % HFP);
  if (threadIdx.x == 0) D.bsum[blockIdx.x] = t % HFP;
}

// divisor x - a (d1 = 1, d0 = -a): q[j] = a^-(j+1) sum_{i>j} num[i] a^i, rem = num[0] + a q[0].
// The block's suffix sums by wave shuffles; the carry (the aggregates of every block after this
// one, from the sums phase) reduced in the same pass: ONE barrier per block.
__global__ __launch_bounds__(SCAN_T) void lin_scan_apply_kernel(LinDivs L, const uint8_t* __restrict__ S) {
  const LinDiv& D = L.d[blockIdx.y];
  if ((int)blockIdx.x >= D.nb) return;
  const uint8_t* num = D.num;
  const uint64_t nl = D.nl;
  uint8_t* q = D.q;
  const uint32_t a = S[D.aslot];
  uint32_t pw[16], ipw[16];
  pw[0] = ipw[0] = 1;
  const uint32_t ai = hinv(a);
#pragma unroll
  for (int j = 1; j < 16; j++) { pw[j] = pw[j - 1] * a % HFP; ipw[j] = ipw[j - 1] * ai % HFP; }
  // thread owns SCAN_E = 16 consecutive elements [base, base + 16): base % 16 = 0
  const uint64_t base = (uint64_t)blockIdx.x * SCAN_B + (uint64_t)threadIdx.x * SCAN_E;
  uint32_t nb8[4] = {0, 0, 0, 0};
  if (D.vec) {
    load16(num, nl, base, nb8);
  } else {
#pragma unroll
    for (int k = 0; k < 16; k++)
      if (base + k < nl) nb8[k >> 2] |= (uint32_t)num[base + k] << (8 * (k & 3));
  }
  uint32_t w[SCAN_E];
  uint32_t tot = 0;
#pragma unroll
  for (int k = 0; k < SCAN_E; k++) {
    const uint64_t i = base + k;
    w[k] = (i > 0) ? hmod(((nb8[k >> 2] >> (8 * (k & 3))) & 0xFFu) * pw[k]) : 0u;   // (<= 255 x 16)
    tot += w[k];
  }
  uint32_t c = 0;
  for (int b = (int)blockIdx.x + 1 + (int)threadIdx.x; b < D.nb; b += SCAN_T) c += D.bsum[b];
  const uint32_t suf = wave_suffix(tot);   // this lane's chunk and every later lane's
  const uint32_t cw = wave_sum(c % HFP);
  __shared__ uint32_t ws[2][SCAN_T / 64];
  const int wv = (int)(threadIdx.x >> 6);
  if ((threadIdx.x & 63) == 0) {
    ws[0][wv] = suf;   // lane 0: the wave's total
    ws[1][wv] = cw;
  }
  __syncthreads();
  uint32_t run = suf - tot;   // sum of w over elements after this thread's chunk
#pragma unroll
  for (int u = 0; u < SCAN_T / 64; u++) run += (u > wv ? ws[0][u] : 0u) + ws[1][u];
  const uint64_t ql = nl - 1;
  uint32_t o[4] = {0, 0, 0, 0};
#pragma unroll
  for (int k = SCAN_E - 1; k >= 0; k--) {
    const uint64_t j = base + k;   // run = sum_{i > j} w_i
    if (j < ql) {
      const uint32_t v = a == 0 ? (uint32_t)num[j + 1] : run % HFP * ipw[(k + 1) & 15] % HFP;
      o[k >> 2] |= v << (8 * (k & 3));
      if (j == 0 && (num[0] + a * v) % HFP) atomicOr(D.flag, 1u);
    }
    run += w[k];
  }
  if (D.vec && base + 16 <= ql) {
    *reinterpret_cast<uint4*>(q + base) = make_uint4(o[0], o[1], o[2], o[3]);
  } else {
#pragma unroll
    for (int k = 0; k < 16; k++)
      if (base + k < ql) q[base + k] = (uint8_t)(o[k >> 2] >> (8 * (k & 3)));
  }
}

// The quotient bytes of one 4096-coefficient chunk of a division by x - av, from the chunk's
// numerator bytes (nb8: this thread's E, packed), the thread's powers pt[k] = av^(base + k) and
// ipt[k] = av^-(base + k + 1) (exponents mod 16), and the carry (this thread's part of the sum of
// every later chunk's aggregate, < 17) -- lin_scan_apply_kernel's work on packed coefficients,
// shared by the one-launch divisions.  T threads of E coefficients each: T E = 4096.
template <int T, int E>
__device__ __forceinline__ void lin_div_finish(const LcArgs& a, const LinDiv& D, const uint32_t (&cf)[LC_MAX],
                                               uint32_t sc, uint32_t av, uint64_t base, uint64_t nl,
                                               const uint32_t (&nb8)[E / 4], const uint32_t (&pt)[E],
                                               const uint32_t (&ipt)[E], uint32_t carry) {
  static_assert(T * E == SCAN_B && E % 4 == 0, "a scan chunk");
  uint32_t w[E], tot = 0;
#pragma unroll
  for (int k = 0; k < E; k++) {
    w[k] = base + k > 0 ? hmod(((nb8[k >> 2] >> (8 * (k & 3))) & 0xFFu) * pt[k]) : 0u;
    tot += w[k];
  }
  // a = 0: q[j] = num[j + 1], which for the thread's last coefficient is the next thread's first
  // (lane shuffle / LDS across waves) or, for the block's last thread, the next chunk's first
  // coefficient (recomputed from the terms: nt byte loads, that thread only)
  __shared__ uint32_t first[T / 64 + 1];
  const int lane = (int)(threadIdx.x & 63), wv = (int)(threadIdx.x >> 6);
  uint32_t nxt = __shfl_down(nb8[0] & 0xFFu, 1, 64);
  if (av == 0) {   // (uniform)
    if (lane == 0) first[wv] = nb8[0] & 0xFFu;
    if (threadIdx.x == T - 1) {
      const uint64_t i = base + E;
      uint32_t s = 0;
      for (int u = 0; u < a.nt; u++) s += i < a.len[u] ? cf[u] * a.p[u][i] : 0u;
      first[T / 64] = i < nl ? hmod(hmod(s) * sc) : 0u;
    }
  }
  // suffix sums: lanes, waves, then the later chunks' carry -- one barrier
  const uint32_t suf = wave_suffix(tot);                 // (<= 64 x E x 16)
  const uint32_t cw = hmod(wave_sum(carry));             // (the wave sum <= 64 x 16)
  __shared__ uint32_t ws[2][T / 64];
  if (lane == 0) {
    ws[0][wv] = suf;
    ws[1][wv] = cw;
  }
  __syncthreads();
  if (av == 0 && lane == 63) nxt = first[wv + 1];
  uint32_t run = suf - tot;
#pragma unroll
  for (int u = 0; u < T / 64; u++) run += (u > wv ? ws[0][u] : 0u) + ws[1][u];
  run = hmod(run);   // (<= 4096 x 16 + T / 64 x 16 < 69632)
  const uint64_t ql = nl - 1;
  uint32_t o[E / 4] = {};
#pragma unroll
  for (int k = E - 1; k >= 0; k--) {
    const uint64_t j = base + k;   // run = sum_{i > j} w_i (mod 17: < 17 + (E - 1) x 16 below)
    if (j < ql) {
      const uint32_t nx = k == E - 1 ? nxt : (nb8[(k + 1) >> 2] >> (8 * ((k + 1) & 3))) & 0xFFu;
      const uint32_t v = av == 0 ? nx : hmod(hmod(run) * ipt[k]);
      o[k >> 2] |= v << (8 * (k & 3));
      if (j == 0 && ((nb8[0] & 0xFFu) + av * v) % HFP) atomicOr(D.flag, 1u);
    }
    run += w[k];
  }
  uint8_t* q = D.q;
  if (D.vec && base + E <= ql) {
    if constexpr (E == 16) *reinterpret_cast<uint4*>(q + base) = make_uint4(o[0], o[1], o[2], o[3]);
    else *reinterpret_cast<uint2*>(q + base) = make_uint2(o[0], o[1]);
  } else {
#pragma unroll
    for (int k = 0; k < E; k++)
      if (base + k < ql) q[base + k] = (uint8_t)(o[k >> 2] >> (8 * (k & 3)));
  }
}
// av^k and av^-(k + 1) for k < 16 (exponents mod 16: av^16 = 1 for av != 0)
__device__ __forceinline__ void div_powers(uint32_t av, uint32_t (&pw)[16], uint32_t (&ipw)[16]) {
  const uint32_t ai = hinv(av);
  pw[0] = 1;
  ipw[15] = 1;   // av^-16 = av^0
  uint32_t x = ai;
#pragma unroll
  for (int j = 1; j < 16; j++) pw[j] = pw[j - 1] * av % HFP;
#pragma unroll
  for (int j = 0; j < 15; j++) {   // ipw[j] = ai^(j + 1)
    ipw[j] = x;
    x = x * ai % HFP;
  }
}

// Round 5 in ONE launch (PLK_OPT_PROVE_FUSE_DIV): each block forms its 4096-coefficient chunk
// of the numerator in registers (lincomb_scan_kernel's loads), publishes the chunk's aggregate
// as one 64-bit word {epoch, sum}, then reduces the aggregates of every later chunk and finishes
// its quotient bytes as lin_scan_apply_kernel does -- the numerator is never stored or re-read.
// Chunks are taken in REVERSE block order: a block waits only for chunks owned by blocks that
// were dispatched before it (running or done), so the waits cannot deadlock whatever the
// residency.  A wait that still sees a stale word after ~2^22 polls gives up and marks the
// division's remainder word with SCAN_TIMEOUT (reported as an internal error, never a proof).
constexpr uint32_t SCAN_TIMEOUT = 1u << 30;
__global__ __launch_bounds__(SCAN_T) void lincomb_divide_kernel(LcBatch b, LinDivs L, const uint8_t* __restrict__ S,
                                                               unsigned long long* __restrict__ fw0, uint32_t fw_stride,
                                                               uint32_t epoch) {
  const int d = blockIdx.y;
  const LcArgs& a = b.a[d];
  const LinDiv& D = L.d[d];
  const int c = (int)(gridDim.x - 1 - blockIdx.x);   // this block's chunk
  if (c >= D.nb) return;
  unsigned long long* fw = fw0 + (uint64_t)d * fw_stride;
  // (the scalars are uniform: read into SGPRs, so the power tables below cost no VGPRs)
  uint32_t cf[LC_MAX];
#pragma unroll
  for (int t = 0; t < LC_MAX; t++) cf[t] = __builtin_amdgcn_readfirstlane(t < a.nt ? S[a.slot[t]] : 0u);
  const uint32_t sc = __builtin_amdgcn_readfirstlane(S[a.scale]);
  const uint32_t c0 = __builtin_amdgcn_readfirstlane(a.c0 >= 0 ? S[a.c0] : 0u);
  const uint32_t c1 = __builtin_amdgcn_readfirstlane(a.c1 >= 0 ? S[a.c1] : 0u);
  const uint64_t base = (uint64_t)c * SCAN_B + (uint64_t)threadIdx.x * SCAN_E;
  const uint64_t nl = a.out_len;
  uint32_t acc[16];
  lc16_swar(a, cf, c0, c1, base, acc);
  const uint32_t av = __builtin_amdgcn_readfirstlane(S[D.aslot]);
  uint32_t pw[16];
  pw[0] = 1;
#pragma unroll
  for (int j = 1; j < 16; j++) pw[j] = pw[j - 1] * av % HFP;
  // the chunk's numerator coefficients num[base + k] (0 past nl), packed, and the thread's part of
  // the chunk aggregate sum_{i > 0} num[i] a^i ((base + k) mod 16 = k)
  uint32_t nb8[4] = {0, 0, 0, 0}, agg = 0;
#pragma unroll
  for (int k = 0; k < 16; k++) {
    const uint32_t v = base + k < nl ? hmod(hmod(acc[k]) * sc) : 0u;   // (acc <= 16 x 16 x 255 + 32)
    nb8[k >> 2] |= v << (8 * (k & 3));
    if (base + k > 0) agg += v * pw[k];
  }
  // publish the chunk aggregate
  const uint32_t t = scan_block_sum(agg % HFP) % HFP;
  if (threadIdx.x == 0)
    __hip_atomic_store(fw + c, ((unsigned long long)epoch << 32) | t, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  // the aggregates of every later chunk (each word carries its own payload: no fence needed)
  uint32_t carry = 0;
  bool late = false;
  for (int cb = c + 1 + (int)threadIdx.x; cb < D.nb; cb += SCAN_T) {
    unsigned long long v = __hip_atomic_load(fw + cb, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    for (uint32_t it = 0; (uint32_t)(v >> 32) != epoch; it++) {
      if (it == (1u << 22)) { late = true; break; }
      __builtin_amdgcn_s_sleep(1);
      v = __hip_atomic_load(fw + cb, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    carry += (uint32_t)v % HFP;
  }
  if (late) atomicOr(D.flag, SCAN_TIMEOUT);
  uint32_t pw2[16], ipw[16];
  div_powers(av, pw2, ipw);
  lin_div_finish<SCAN_T, SCAN_E>(a, D, cf, sc, av, base, nl, nb8, pw2, ipw, carry % HFP);
}

// Round 5 in ONE launch with no waits (PLK_OPT_PROVE_EVAL_AGG): the scan's chunk aggregates are
// linear in the numerator's terms -- sum_{i in c} W[i] z^i = sc sum_t cf_t sum_{i in c} p_t[i] z^i
// (W = sc sum_t cf_t p_t; the constants sit at i = 0, 1, in chunk 0, which is never a later chunk)
// -- and round 4 already evaluates every term at z.  Its evaluation rows store each term's chunk
// sums (EvArgs::col, 16-byte records of agg[]: one column per term, t_lo / t_mid / t_hi as rows of
// their own; z(omega x) evaluated at z gives z_x's sums at z omega for the second division), so
// this launch forms its chunk of both numerators in registers, reduces the later chunks' records
// against the round-4 coefficients (one v_dot4 per 4 columns) and writes the quotient bytes: the
// numerators are never stored and lin_scan_apply_kernel's launch is gone.  Extra grid rows run
// the commitments that do not wait for round 5, as lincomb_scan_kernel's do.
struct AggMap {
  const uint8_t* agg;        // [chunk][16] column sums (prover memory, written by eval_kernel)
  int8_t col[2][LC_MAX];     // division d, numerator term t -> its agg column (-1: none)
};
// 512 threads of 8 coefficients per 4096-coefficient chunk: twice the waves of the 16-coefficient
// form over the same ~770 chunks (one block each), so more of each block's load -> sum -> scan chain
// overlaps (the chain, not the bytes, bounds this launch)
constexpr int AGG_T = 512, AGG_E = SCAN_B / AGG_T;
__global__ __launch_bounds__(AGG_T) void lincomb_agg_divide_kernel(LcBatch b, LinDivs L, const uint8_t* __restrict__ S,
                                                                  AggMap m, EarlyMsm em) {
  if ((int)blockIdx.y >= em.nd) {   // (uniform) an early commitment row
    __shared__ uint32_t etab[PLK_GROUP_ORDER];
    __shared__ uint32_t wsum[AGG_T / PLK_WAVE];
    __shared__ uint32_t wbad[AGG_T / PLK_WAVE];
    const int r = (int)blockIdx.y - em.nd;
    if (blockIdx.x >= em.X) return;
    (void)msm_log_block<AGG_T>(em.logs, em.arena + (uint64_t)r * em.cstride, em.rl.n[r], blockIdx.x, em.X, (uint32_t)r,
                               em.res + r, em.exp_words, etab, wsum, wbad);
    return;
  }
  const int d = blockIdx.y;
  const LcArgs& a = b.a[d];
  const LinDiv& D = L.d[d];
  const int c = (int)blockIdx.x;
  if (c >= D.nb) return;
  uint32_t cf[LC_MAX];
#pragma unroll
  for (int t = 0; t < LC_MAX; t++) cf[t] = __builtin_amdgcn_readfirstlane(t < a.nt ? S[a.slot[t]] : 0u);
  const uint32_t sc = __builtin_amdgcn_readfirstlane(S[a.scale]);
  const uint32_t c0 = __builtin_amdgcn_readfirstlane(a.c0 >= 0 ? S[a.c0] : 0u);
  const uint32_t c1 = __builtin_amdgcn_readfirstlane(a.c1 >= 0 ? S[a.c1] : 0u);
  const uint64_t base = (uint64_t)c * SCAN_B + (uint64_t)threadIdx.x * AGG_E;
  const uint64_t nl = a.out_len;
  // the later chunks' records: one per thread loaded before the numerator's terms (a division of
  // up to 513 chunks, ~2^21 coefficients, needs no more), the rest after
  const uint4* rec = reinterpret_cast<const uint4*>(m.agg);
  const int cb0 = c + 1 + (int)threadIdx.x;
  const uint4 r0 = cb0 < D.nb ? rec[cb0] : make_uint4(0u, 0u, 0u, 0u);
  uint32_t acc[AGG_E];
  lc_swar<AGG_E / 4>(a, cf, c0, c1, base, acc);
  // column weights K = sc cf_t mod 17 packed as bytes: one v_dot4_u32_u8 per record word
  uint32_t K[4] = {0, 0, 0, 0};
#pragma unroll
  for (int t = 0; t < LC_MAX; t++) {
    const int col = m.col[d][t];
    if (t < a.nt && col >= 0) K[col >> 2] += (cf[t] * sc % HFP) << (8 * (col & 3));
  }
  auto dot = [&](const uint4& r) {   // (<= 4 x 4 x 16 x 16)
    return __builtin_amdgcn_udot4(r.x, K[0], __builtin_amdgcn_udot4(r.y, K[1], 0u, false), false) +
           __builtin_amdgcn_udot4(r.z, K[2], __builtin_amdgcn_udot4(r.w, K[3], 0u, false), false);
  };
  uint32_t carry = dot(r0);
  for (int cb = cb0 + AGG_T; cb < D.nb; cb += AGG_T) carry += dot(rec[cb]) % HFP;
  const uint32_t av = __builtin_amdgcn_readfirstlane(S[D.aslot]);
  uint32_t pw[16], ipw[16];
  div_powers(av, pw, ipw);
  // this thread's coefficients start at base = 0 or 8 (mod 16): its powers from there
  const bool odd = (base & 15u) != 0;
  uint32_t pt[AGG_E], ipt[AGG_E];
#pragma unroll
  for (int k = 0; k < AGG_E; k++) {
    pt[k] = odd ? pw[(k + AGG_E) & 15] : pw[k];
    ipt[k] = odd ? ipw[(k + AGG_E) & 15] : ipw[k];
  }
  uint32_t nb8[AGG_E / 4] = {};
#pragma unroll
  for (int k = 0; k < AGG_E; k++) {
    const uint32_t v = base + k < nl ? hmod(hmod(acc[k]) * sc) : 0u;   // (acc <= 16 x 16 x 255 + 32)
    nb8[k >> 2] |= v << (8 * (k & 3));
  }
  lin_div_finish<AGG_T, AGG_E>(a, D, cf, sc, av, base, nl, nb8, pt, ipt, carry % HFP);
}

// (c) any other divisor: the reference's long division in one workgroup (only reached for
// tiny non-subgroup H, e.g. n = 3).
__global__ __launch_bounds__(256) void divide_general_kernel(const uint8_t* __restrict__ num, uint64_t nl,
                                                             const uint8_t* __restrict__ den, uint64_t dl,
                                                             uint8_t* __restrict__ rem, uint8_t* __restrict__ q,
                                                             uint32_t* rem_flag) {
  for (uint64_t i = threadIdx.x; i < nl; i += blockDim.x) rem[i] = num[i];
  __syncthreads();
  const uint32_t li = hinv(den[dl - 1]);
  for (int64_t i = (int64_t)nl - 1; i >= (int64_t)dl - 1; i--) {
    const uint32_t coeff = rem[i] * li % HFP;
    __syncthreads();
    if (threadIdx.x == 0) q[i - (dl - 1)] = (uint8_t)coeff;
    for (uint64_t j = threadIdx.x; j < dl; j += blockDim.x)
      rem[i - j] = (uint8_t)((rem[i - j] + HFP - coeff * den[dl - 1 - j] % HFP) % HFP);
    __syncthreads();
  }
  const uint64_t rl = dl - 1 < nl ? dl - 1 : nl;
  for (uint64_t i = threadIdx.x; i < rl; i += blockDim.x)
    if (rem[i]) atomicOr(rem_flag, 1u);
}

// ------------------------------------------------------------------ trimmed lengths
// one block per buffer: index + 1 of the last non-zero byte, at least 1 (src/poly.h:20-24)
// dst | TRIM_ANY: write 1 to the word if any byte is non-zero (a flag), leave it otherwise
constexpr int TRIM_ANY = 1 << 16;
struct TrimArgs {
  const uint8_t* p[11];
  uint64_t len[11];
  int dst[11];
};
// ------------------------------------------------------------------ scalar programs
// Rounds 4 and 5's scalar programs, run by one thread after the evaluations at z: the whole
// 128-byte file is read at once (eight 16-byte loads in flight, not a chain of dependent byte
// loads), the derived slots are stored at the end.  tz = t(z) (S_TZ: the caller may have just
// stored it itself).
__device__ void scalars_r45(uint8_t* S, uint32_t tz) {
  uint32_t W[NSLOT / 4];
#pragma unroll
  for (int i = 0; i < NSLOT / 16; i++) {
    const uint4 q = reinterpret_cast<const uint4*>(S)[i];
    W[4 * i] = q.x; W[4 * i + 1] = q.y; W[4 * i + 2] = q.z; W[4 * i + 3] = q.w;
  }
  auto g = [&](int s) -> uint32_t { return (W[s >> 2] >> (8 * (s & 3))) & 0xFFu; };
  const uint32_t al = g(S_ALPHA), be = g(S_BETA), ga = g(S_GAMMA), z = g(S_Z), v = g(S_V);
  const uint32_t az = g(S_AZ), bz = g(S_BZ), cz = g(S_CZ), s1 = g(S_S1Z), s2 = g(S_S2Z);
  const uint32_t zw = g(S_ZWZ), l1 = g(S_L1Z);
  const uint32_t ab = az * bz % HFP;
  // src/plonk.h:547-556: r_2 scale
  const uint32_t x1 = (az + be * z + ga) % HFP;
  const uint32_t x2 = (bz + be * g(S_K1) % HFP * z + ga) % HFP;
  const uint32_t x3 = (cz + be * g(S_K2) % HFP * z + ga) % HFP;
  const uint32_t r2 = x1 * x2 % HFP * x3 % HFP * al % HFP;
  // src/plonk.h:569: r_4 scale
  const uint32_t r4 = l1 * g(S_ALPHA2) % HFP;
  const uint32_t r24 = (r2 + r4) % HFP;
  // src/plonk.h:559-566: r_3
  const uint32_t bzw = be * zw % HFP;
  const uint32_t y1 = (az + be * s1 + ga) % HFP, y2 = (bz + be * s2 + ga) % HFP;
  const uint32_t r3 = y1 * y2 % HFP * al % HFP;
  const uint32_t r3b = r3 * bzw % HFP;   // r_3 scale times the s_sigma_3 factor
  // r_z = r(z) (src/plonk.h:571) from the evaluations of r(x)'s terms: evaluation is a ring
  // homomorphism, so sum_i c_i p_i(z) = (sum_i c_i p_i)(z) mod 17
  const uint32_t cs[6] = {ab, az, bz, cz, r24, r3b};
  const uint32_t ez[6] = {g(S_QMZ), g(S_QLZ), g(S_QRZ), g(S_QOZ), g(S_ZXZ), g(S_P3Z)};
  uint32_t rz = 0;
  for (int i = 0; i < 6; i++) rz += cs[i] * ez[i];
  rz %= HFP;
  // constant term of w_z(x), src/plonk.h:584-603
  uint32_t c = hneg(tz);
  c += v * hneg(rz);
  c += g(S_V2) * hneg(az);
  c += g(S_V3) * hneg(bz);
  c += g(S_V4) * hneg(cz);
  c += g(S_V5) * hneg(s1);
  c += g(S_V6) * hneg(s2);
  S[S_AB] = (uint8_t)ab;
  S[S_R24] = (uint8_t)r24;
  S[S_BZW] = (uint8_t)bzw;
  S[S_R3] = (uint8_t)r3;
  S[S_R3B] = (uint8_t)r3b;
  for (int i = 0; i < 6; i++) S[S_VAB + i] = (uint8_t)(v * cs[i] % HFP);   // w_z(x) takes v r(x) term by term
  S[S_RZ] = (uint8_t)rz;
  S[S_NEGZWZ] = (uint8_t)hneg(zw);
  S[S_W0] = (uint8_t)(c % HFP);
}

// The scalar file (challenges, constants, blinding scalars) travels as a kernel argument, and
// the same launch clears status words [st0, st1): no pageable host->device copy (each of those
// stalls the host ~20 us) before the first compute kernel.  (prep_kernel does both itself.)
__global__ void scalars_init_kernel(SlotFile f, uint8_t* __restrict__ S, uint32_t* __restrict__ stat, int st0,
                                    int st1) {
  const int t = threadIdx.x;
  if (t < NSLOT) S[t] = f.b[t];
  if (t >= st0 && t < st1) stat[t] = 0;
}

// 9 commitments (the points in the MSM result records) + 7 evaluations -> PROOF
// (src/plonk.h:24-41: 9 x G1 {x, y, infinite}, then a_z b_z c_z s1_z s2_z r_z z_omega_z)
// The proof bytes and the status words go straight to mapped pinned host memory (`host`:
// 64 proof bytes, then NSTAT words), so the call's end is one stream synchronize and no
// device->host copies.
// The trimmed lengths (formerly a kernel of their own) and the packing in ONE block of 1024 threads, after
// the MSM (which runs over the committed length and does not need them): wave w < ntrim finds
// buffer w's last non-zero byte from the top, 1 KB per step (16 bytes per lane, the highest
// non-zero lane by ballot); the remaining waves OR the remainder-vote bytes (TRIM_ANY).
#ifndef PLK_DIAG_PACK_ONLY
#define PLK_DIAG_PACK_ONLY 0   // timing builds only: 1 skips the trimmed-length scans (wrong status words)
#endif
constexpr int PACK_T = 1024;
static_assert(NSTAT <= 64 && 34 <= 64, "trim_pack_kernel: wave 0 writes the status words, the last wave the proof");
__global__ __launch_bounds__(PACK_T) void trim_pack_kernel(TrimArgs a, int nt, const PlkMsmResult* __restrict__ res,
                                                           const uint8_t* __restrict__ S, uint32_t* __restrict__ stat,
                                                           uint8_t* __restrict__ host, uint32_t seq) {
  const int t = threadIdx.x, wv = t >> 6, lane = t & 63;
  const int ntrim = PLK_DIAG_PACK_ONLY ? 0 : nt > 0 && (a.dst[nt - 1] & TRIM_ANY) ? nt - 1 : nt;   // the vote buffer comes last
  // the proof bytes do not depend on the trimmed lengths: the last waves load and send them to
  // the host first, so their round trips overlap the scans below
  if (wv == PACK_T / 64 - 1) {
    const int ev[7] = {S_AZ, S_BZ, S_CZ, S_S1Z, S_S2Z, S_RZ, S_ZWZ};
    if (lane < 27) host[lane] = res[lane / 3].g1[lane % 3];
    else if (lane < 34) host[lane] = S[ev[lane - 27]];
  }
  __shared__ uint32_t got[11];
  if (t < 11) got[t] = 0;
  __syncthreads();
  if (wv < ntrim) {
    const uint8_t* p = a.p[wv];
    for (uint64_t hi = a.len[wv]; hi > 0;) {
      const uint64_t lo = hi > 1024 ? hi - 1024 : 0;
      uint32_t found = 0;   // index + 1 of this lane's highest non-zero byte
#pragma unroll
      for (int k = 15; k >= 0; k--) {   // lane l: bytes hi - 16 (l + 1) .. hi - 16 l - 1
        const int64_t i = (int64_t)hi - 16 * (lane + 1) + k;
        const bool nz = i >= (int64_t)lo && p[i < (int64_t)lo ? lo : i] != 0;
        found = (!found && nz) ? (uint32_t)(i + 1) : found;
      }
      const unsigned long long bal = __ballot(found != 0);
      if (bal) {
        const uint32_t v = __shfl(found, __ffsll(bal) - 1, 64);   // lowest lane = highest bytes
        if (lane == 0) got[wv] = v;
        break;
      }
      hi = lo;
    }
  } else if (ntrim < nt) {
    const uint8_t* p = a.p[nt - 1];
    const uint64_t n = a.len[nt - 1];
    uint32_t any = 0;
    for (uint64_t i = (uint64_t)(t - ntrim * 64); i < n; i += (uint64_t)(PACK_T - ntrim * 64)) any |= p[i];
    if (any) got[nt - 1] = 1;
  }
  __syncthreads();
  if (t < nt) {
    const int d = a.dst[t];
    if (d & TRIM_ANY) {
      if (got[t]) stat[d & ~TRIM_ANY] = 1u;
    } else {
      stat[d] = got[t] ? got[t] : 1u;   // at least 1 (src/poly.h:20-24)
    }
  }
  __syncthreads();   // the stat words written above, visible to the block
  if (t < NSTAT) ((uint32_t*)(host + 64))[t] = stat[t];
  // the call's completion word (host bytes 60..63) last: every writer's bytes are visible to the
  // host before it (a system-scope fence in the two waves that wrote host bytes, then the
  // barrier), so the host can poll it instead of waiting for the stream (finish())
  if (wv == 0 || wv == PACK_T / 64 - 1) __threadfence_system();
  __syncthreads();
  if (t == 0) __hip_atomic_store((uint32_t*)(host + 60), seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

// The commitments, the trimmed lengths and the packing in ONE launch (the prover's SRS in log
// form, PLK_OPT_PROVE_PACK_FUSE): rows y < nrows of the grid are the log-form MSMs of arena rows
// row0 + y (all 9, or only w_z and w_z_omega when the other 7 ran inside round 5's scan launch,
// PLK_OPT_PROVE_EARLY_COMMITS); row nrows scans the trimmed-length buffers (block x < nt: buffer x, 4 KB per step from the
// top; the vote buffer's block ORs its bytes) while the MSM rows stream.  Every finished record
// and every trim block then arrives on `done`; the last arrival (one thread) packs the proof and
// the status words into the mapped host buffer and writes the completion word, as
// trim_pack_kernel does -- its launch and its scan latency leave the proof's tail.
constexpr int CP_T = 256;
__global__ __launch_bounds__(CP_T) void commit_pack_kernel(const uint8_t* __restrict__ logs, const uint8_t* arena,
                                                           uint64_t cstride, MsmRowLens rl, PlkMsmResult* res,
                                                           const uint32_t* __restrict__ exp_words, int row0, int nrows,
                                                           TrimArgs a, int nt, const uint8_t* __restrict__ S,
                                                           uint32_t* stat, uint8_t* __restrict__ host, uint32_t seq,
                                                           uint32_t* done) {
  __shared__ uint32_t etab[PLK_GROUP_ORDER];
  __shared__ uint32_t wsum[CP_T / PLK_WAVE];
  __shared__ uint32_t wbad[CP_T / PLK_WAVE];
  bool arrive = false;
  if ((int)blockIdx.y < nrows) {   // arena row / record row0 + y
    const int r = row0 + (int)blockIdx.y;
    arrive = msm_log_block<CP_T>(logs, arena + (uint64_t)r * cstride, rl.n[r], blockIdx.x, gridDim.x, (uint32_t)r, res + r,
                                 exp_words, etab, wsum, wbad);
  } else {
    const int x = (int)blockIdx.x;
    if (x >= nt) return;   // (uniform)
    const uint8_t* p = a.p[x];
    const uint64_t len = a.len[x];
    const int d = a.dst[x];
    if (d & TRIM_ANY) {   // the remainder votes: any non-zero byte
      uint32_t any = 0;
      for (uint64_t i = threadIdx.x; i < len; i += CP_T) any |= p[i];
      any = __syncthreads_or(any != 0);
      if (threadIdx.x == 0 && any) stat[d & ~TRIM_ANY] = 1u;
    } else {               // index + 1 of the last non-zero byte, at least 1 (src/poly.h:20-24)
      uint32_t found = 0;
      for (uint64_t hi = len; hi > 0;) {
        const uint64_t lo = hi > 16 * CP_T ? hi - 16 * CP_T : 0;
#pragma unroll
        for (int k = 15; k >= 0; k--) {   // thread t: bytes hi - 16 (t + 1) .. hi - 16 t - 1
          const int64_t i = (int64_t)hi - 16 * ((int64_t)threadIdx.x + 1) + k;
          const bool nz = i >= (int64_t)lo && p[i < (int64_t)lo ? lo : i] != 0;
          found = (!found && nz) ? (uint32_t)(i + 1) : found;
        }
        found = plk_block_max(found);
        if (found) break;   // (uniform: the block's maximum)
        hi = lo;
      }
      if (threadIdx.x == 0) stat[d] = found ? found : 1u;
    }
    arrive = threadIdx.x == 0;
  }
  if (!arrive) return;
  // this record's point / this trim's word is written: release it, then arrive
  __threadfence();
  if (atomicAdd(done, 1u) != (uint32_t)nrows + (uint32_t)nt - 1u) return;
  __threadfence();   // (acquire: every other arrival's writes are visible)
  *done = 0;         // re-armed for the next proof
  const int ev[7] = {S_AZ, S_BZ, S_CZ, S_S1Z, S_S2Z, S_RZ, S_ZWZ};
  for (int i = 0; i < 27; i++) host[i] = res[i / 3].g1[i % 3];
  for (int i = 0; i < 7; i++) host[27 + i] = S[ev[i]];
  for (int i = 0; i < NSTAT; i++) ((uint32_t*)(host + 64))[i] = __hip_atomic_load(stat + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __threadfence_system();
  __hip_atomic_store((uint32_t*)(host + 60), seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

// ------------------------------------------------------------------ stage A (circuit)
// constraints_satisfy (src/constraints.h:145-171) and copy_constraints_to_roots
// (src/plonk.h:141-160): one thread per gate.
__global__ void circuit_check_kernel(const uint8_t* __restrict__ cir, uint64_t n, const uint8_t* __restrict__ h3,
                                     uint8_t* __restrict__ vals, uint32_t* __restrict__ stat) {
  // cir: q_m q_l q_r q_o q_c | copies a,b,c as (type, index) pairs | a b c   (n each / 2n each)
  // vals (11 x n): a b c q_o q_m q_l q_r q_c sigma1 sigma2 sigma3
  const uint8_t *qm = cir, *ql = cir + n, *qr = cir + 2 * n, *qo = cir + 3 * n, *qc = cir + 4 * n;
  const uint8_t* cp = cir + 5 * n;
  const uint8_t *wa = cir + 11 * n, *wb = cir + 12 * n, *wc = cir + 13 * n;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    const uint32_t a = wa[i], b = wb[i], c = wc[i];
    const uint32_t lhs = (ql[i] * a + qr[i] * b + qo[i] * c + qm[i] * (a * b % HFP) + qc[i]) % HFP;
    if (lhs) atomicMin(&stat[ST_GATE], (uint32_t)i + 1);
    vals[0 * n + i] = (uint8_t)a;
    vals[1 * n + i] = (uint8_t)b;
    vals[2 * n + i] = (uint8_t)c;
    vals[3 * n + i] = qo[i];
    vals[4 * n + i] = qm[i];
    vals[5 * n + i] = ql[i];
    vals[6 * n + i] = qr[i];
    vals[7 * n + i] = qc[i];
    for (int k = 0; k < 3; k++) {
      const uint32_t type = cp[2 * (k * n + i)], idx = cp[2 * (k * n + i) + 1];
      uint8_t s = 0;
      if (type > 2 || idx == 0 || idx > n) atomicMin(&stat[ST_COPY], (uint32_t)(k * n + i) + 1);
      else s = h3[type * n + (idx - 1)];   // h | k1_h | k2_h
      vals[(8 + k) * n + i] = s;
    }
  }
}

// interpolate_at_h (src/plonk.h:162-195): out[v][r] = sum_c Hinv[r][c] vals[v][c] (matrix_mul,
// src/matrix.h:81), batched over nv vectors; one thread per (vector, row).
__global__ void interpolate_kernel(const uint8_t* __restrict__ hinvm, uint64_t n, const uint8_t* __restrict__ vals,
                                   int nv, uint8_t* const* __restrict__ outs) {
  const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= (uint64_t)nv * n) return;
  const uint64_t v = t / n, r = t % n;
  uint32_t acc = 0;
  for (uint64_t c = 0; c < n; c++) {
    acc += hinvm[r * n + c] * vals[v * n + c];
    if ((c & 0xFFFF) == 0xFFFF) acc %= HFP;
  }
  outs[v][r] = (uint8_t)(acc % HFP);
}

// Round 2 grand product (src/plonk.h:326-359).  The s_sigma evaluations at omega^(i-1) take
// at most 16 distinct points, evaluated by all threads first; the prefix product is serial
// (n is the size of a subgroup of GF(17)*: <= 16).
__global__ void grand_product_kernel(const uint8_t* __restrict__ vals, uint64_t n, const uint8_t* const* polys,
                                     const uint8_t* __restrict__ S, uint8_t* __restrict__ acc) {
  __shared__ uint32_t ev[3][16];
  const uint32_t om = S[S_OMEGA];
  for (int t = threadIdx.x; t < 48; t += blockDim.x) {
    const int k = t / 16, j = t % 16;
    const uint32_t x = hpow_d(om, j);
    const uint8_t* p = polys[8 + k];   // s_sigma_1..3
    uint32_t y = 0;
    for (int64_t i = (int64_t)n - 1; i >= 0; i--) y = (y * x + p[i]) % HFP;
    ev[k][j] = y;
  }
  __syncthreads();
  if (threadIdx.x != 0) return;
  const uint32_t be = S[S_BETA], ga = S[S_GAMMA], k1 = S[S_K1], k2 = S[S_K2];
  uint32_t a = 1;
  acc[0] = 1;
  for (uint64_t i = 1; i < n; i++) {
    const uint32_t wa = vals[i - 1], wb = vals[n + i - 1], wc = vals[2 * n + i - 1];
    // hf_pow(omega, i-1) = omega^((i-1) mod 16): OMEGA = 4 is a unit
    const uint32_t j = (uint32_t)((i - 1) & 15);
    const uint32_t op = hpow_d(om, j);
    const uint32_t den = (wa + be * op + ga) % HFP * ((wb + be * (k1 * op % HFP) + ga) % HFP) % HFP *
                         ((wc + be * (k2 * op % HFP) + ga) % HFP) % HFP;
    const uint32_t e1 = ev[0][j], e2 = ev[1][j], e3 = ev[2][j];
    const uint32_t num = (wa + be * e1 + ga) % HFP * ((wb + be * e2 + ga) % HFP) % HFP * ((wc + be * e3 + ga) % HFP) % HFP;
    a = a * (den * hinv(num) % HFP) % HFP;
    acc[i] = (uint8_t)a;
  }
}

__global__ void unit_vector_kernel(uint8_t* v, uint64_t n) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
    v[i] = i == 0 ? 1 : 0;
}

// ------------------------------------------------------------------ host side
uint8_t h_pow(uint32_t b, uint64_t e) {
  uint32_t r = 1;
  b %= HFP;
  while (e) {
    if (e & 1) r = r * b % HFP;
    b = b * b % HFP;
    e >>= 1;
  }
  return (uint8_t)r;
}

}  // namespace

// ------------------------------------------------------------------ prover object
struct plk_prover {
  size_t n = 0;
  size_t srs_len = 0;
  bool srs_irregular = false;
  // Z_H shape (host analysis of the trimmed divisor)
  size_t zh_len = 0;
  int zh_kind = 0;   // 0 binomial L x^m + c, 1 general
  uint32_t zh_lead = 1, zh_c = 0;
  bool have_circuit_tables = false;
  // device memory (one allocation, carved)
  uint8_t* mem = nullptr;
  size_t mem_bytes = 0;
  uint8_t *d_srs = nullptr, *d_zh = nullptr, *d_h3 = nullptr, *d_hinv = nullptr;
  uint8_t* d_S = nullptr;          // scalar file
  uint32_t* d_stat = nullptr;      // status words
  uint32_t* d_tick = nullptr;      // eval arrival words (zeroed at create, re-armed by eval_kernel)
  uint8_t* d_rem = nullptr;        // Z_H division: one remainder vote per block
  int lin_sum = 0;                 // round 3: a q_l + b q_r + c q_o computed as one sum (in AQL)
  int t2_sum = 0;                  // round 3: (a b) q_m + t_2 computed as one sum (in T2)
  uint64_t rem_blocks = 0;
  uint32_t* d_bsum = nullptr;      // scan block sums
  uint8_t* d_agg = nullptr;        // round 4's chunk aggregates of round 5's numerator terms [chunk][16]
  unsigned long long* d_scanw = nullptr;   // lincomb_divide_kernel's chunk words {epoch, sum}
  uint32_t scanw_stride = 0;       // words per division
  uint32_t scan_epoch = 0;         // launches of lincomb_divide_kernel so far (0: none)
  PlkMsmResult* d_res = nullptr;   // 9 MSM records
  uint8_t* d_srs_log = nullptr;    // the SRS in log form (srs_log_kernel), valid when !srs_irregular
  const uint32_t* exp_words = nullptr;   // the group's EXP words on this prover's device
  int early_rows = 0;              // commitments of this call already run by round 5's scan launch
  uint32_t* d_srs_flag = nullptr;  // srs_log_kernel's irregular flag
  uint32_t* d_done = nullptr;      // commit_pack_kernel's arrival word (re-armed by its last arrival)
  uint8_t* arena = nullptr;        // [9][cstride] committed polynomials
  size_t cstride = 0, cmax = 0;
  uint8_t* d_polys[13] = {};       // stage-A outputs (circuit path)
  uint8_t* d_cir = nullptr;        // circuit upload
  uint8_t* d_vals = nullptr;       // 11 x n values to interpolate
  uint8_t** d_outs = nullptr;      // device array of the 13 poly pointers
  // intermediates
  uint8_t *blA, *blB, *blC, *zB, *AB, *ABQM, *AQL, *BQR, *CQO, *A2, *B2, *C2, *T2a, *T2b, *T2, *A3, *B3, *C3, *ZW,
      *T3a, *T3b, *T3, *Z1, *T4, *NUM, *TX, *P3, *W, *ZZ, *REMT, *ACCV, *E0;
  void* work = nullptr;
  size_t work_bytes = 0;
  hipStream_t st = nullptr;
  hipEvent_t ev = nullptr;         // cross-stream hand-offs of the strong-scaled proof entry points
  // mapped pinned host memory: 64 proof bytes + NSTAT status words (trim_pack_kernel)
  uint8_t* h_res = nullptr;
  uint8_t* d_res_host = nullptr;   // its device address
  uint32_t seq = 0;                // calls so far: trim_pack_kernel's completion word
  // preprocessed circuit (plk_prover_preprocess): the round-3 forward transforms of the fixed
  // polynomials q_o q_m q_l q_r s_sigma_3 l_1_x (PlkPolyMulJob::bt), for the addresses given
  struct Fixed {
    const uint8_t* src = nullptr;   // the d_polys entry it was computed from
    uint32_t* t = nullptr;          // 2^k words
    int k = 0, field = -1;
  } fix[13];
  uint32_t* fix_mem = nullptr;
  // the device of this prover's memory and stream (a helper may live on another GPU)
  int dev = 0;
  // one proof over several GPUs from C (plk_prover_attach_helpers): helper provers on further
  // entries of the plk_init_devices list compute round 3's t_2 / t_3 chains; their products land
  // in rx[] on this device (hipMemcpyPeerAsync on the helper's stream, then its ev_done)
  int nhelp = 0;
  plk_prover* help[2] = {nullptr, nullptr};
  int help_mask[2] = {0, 0};
  uint8_t* rx_mem = nullptr;
  uint8_t* rx[2] = {nullptr, nullptr};   // received t_2, t_3 (plk_prover_chain_bytes each)
  hipEvent_t ev_in = nullptr;            // recorded on st before the helpers start: the inputs are there
  // as a helper on another device: its copies of the 7 input polynomials it reads
  uint8_t* hin = nullptr;
  hipEvent_t ev_done = nullptr;          // (helper's device) its products have reached the proving device
  // plk_prover_rounds_dev as a captured HIP graph (PLK_OPT_PROVE_GRAPH, rounds_graph): replayed
  // while the inputs' addresses, the preprocessed transforms (fix_gen) and every option are the
  // ones it was captured with; per call the first kernel's scalar file and the last kernel's
  // completion word are set as node parameters
  hipGraph_t g = nullptr;
  hipGraphExec_t gx = nullptr;
  hipGraphNode_t g_first = nullptr, g_last = nullptr;
  int g_first_arg = -1, g_first_n = 0;
  const uint8_t* g_pl[13] = {};
  bool g_pre = false;
  uint32_t fix_gen = 0, g_fix_gen = 0;
  int64_t g_opt[PLK_OPT_COUNT] = {};
  uint32_t g_seq = 0;              // the completion word the graph's last kernel writes
  SlotFile g_sf{};                 // the scalar file its first kernel holds
  // plk_prover_profile_dev: events around the launch sequence [0] .. [5] and round 3's two product
  // batches ([1]-[2], [3]-[4]: every NTT pass kernel of the proof), recorded only while tev_on
  hipEvent_t tev[6] = {};
  bool tev_on = false;
};

namespace {

// upper-bound lengths of every polynomial of rounds 1-5 for n gates and |Z_H| = lz
struct Lens {
  uint64_t n, lz, la, lzx, lab, labqm, lq1, lt1, l2a, l2b, l2, lzw, l3, lz1, lt4, lnum, lq, ltx, lr3, lrx, lw, lwq,
      lzz, lwo;
};
Lens lens_for(uint64_t n, uint64_t lz) {
  Lens L{};
  L.n = n;
  L.lz = lz;
  L.la = std::max<uint64_t>(lz + 1, n);          // a_x, b_x, c_x
  L.lzx = std::max<uint64_t>(lz + 2, n);         // z_x
  L.lab = 2 * L.la - 1;                          // a_x b_x
  L.labqm = L.lab + n - 1;                       // (a_x b_x) q_m
  L.lq1 = L.la + n - 1;                          // a_x q_l, ...
  L.lt1 = std::max(L.labqm, L.lq1);
  L.l2a = 2 * L.la - 1;                          // A2 B2
  L.l2b = L.l2a + L.la - 1;                      // (A2 B2) C2
  L.l2 = L.l2b + L.lzx - 1;                      // ... z_x
  L.lzw = L.lzx;
  L.l3 = L.l2b + L.lzw - 1;
  L.lz1 = L.lzx;
  L.lt4 = L.lz1 + n - 1;
  L.lnum = std::max(std::max(L.lt1, L.l2), std::max(L.l3, L.lt4));
  // quotient by Z_H (len lz)
  L.ltx = L.lnum >= lz ? L.lnum - lz + 1 : 1;
  L.lr3 = L.lzx + n - 1;                         // z_x * (s_sigma_3 scaled)
  L.lrx = std::max(std::max<uint64_t>(n, L.lzx), L.lr3);
  const uint64_t p = n + 2;
  const uint64_t lhi = L.ltx > 2 * p ? L.ltx - 2 * p : 1;
  L.lw = std::max(std::max<uint64_t>(p, lhi), std::max(L.lrx, std::max<uint64_t>(L.la, n)));
  L.lwq = L.lw >= 2 ? L.lw - 1 : 1;
  L.lzz = L.lzx;
  L.lwo = L.lzz >= 2 ? L.lzz - 1 : 1;
  return L;
}

// SURVEY 8(d)'s algorithmic bytes of rounds 1-5 (plk_prover_alg_bytes): the reference's ops as it
// calls them (src/plonk.h:277-621), each at its 8(d) figure -- the 17 poly_mul at la + lb + (la + lb
// - 1) bytes (its own association, ((A2 B2) C2) z), the 9 srs_eval_at_s at 4 B per point, the 3
// poly_divide at numerator + divisor read and quotient + remainder written, the 9 poly_eval at z
// (src/plonk.h:527-533, 567, 574) at one read of the polynomial.  The reference's lincombs (poly_add /
// poly_scale chains) are not counted: a lower bound on any implementation's traffic.
uint64_t alg_bytes_for(const Lens& L) {
  auto pm = [](uint64_t a, uint64_t b) { return a + b + (a + b - 1); };
  const uint64_t n = L.n, lz = L.lz, part = n + 2;
  const uint64_t lmid = L.ltx > part ? std::min<uint64_t>(part, L.ltx - part) : 1;
  const uint64_t lhi = L.ltx > 2 * part ? L.ltx - 2 * part : 1;
  uint64_t s = 3 * pm(2, lz) + pm(3, lz);                                        // rounds 1-2 blindings
  s += pm(L.la, L.la) + pm(L.lab, n) + 3 * pm(L.la, n);                          // a b, (a b) q_m, a q_l ..
  s += 2 * pm(L.la, L.la) + 2 * pm(L.l2a, L.la) + pm(L.l2b, L.lzx) + pm(L.l2b, L.lzw);   // t_2, t_3
  s += pm(L.lz1, n) + pm(L.lzx, n);                                              // Z1 l_1, z_x s_sigma_3
  s += 4 * (3 * L.la + L.lzx + std::min<uint64_t>(part, L.ltx) + lmid + lhi + L.lwq + L.lwo);   // commits
  s += (L.lnum + lz + L.ltx + (lz - 1)) + (L.lw + 2 + L.lwq + 1) + (L.lzz + 2 + L.lwo + 1);     // divisions
  s += 3 * L.la + 2 * n + L.ltx + L.lzw + n + L.lrx;                             // evaluations at z
  return s;
}

struct Bump {
  size_t off = 0;
  size_t take(size_t bytes) {
    const size_t o = off;
    off += (bytes + 255) & ~(size_t)255;
    return o;
  }
};

LcArgs make_lc(std::initializer_list<std::pair<const uint8_t*, uint64_t>> terms, std::initializer_list<int> slots,
               int c0, int c1, int scale, int twist, uint8_t* out, uint64_t out_len) {
  LcArgs a{};
  int t = 0;
  for (const auto& pr : terms) {
    if (t < LC_MAX) { a.p[t] = pr.first; a.len[t] = pr.second; }
    t++;
  }
  int s = 0;
  for (int sl : slots) {
    if (s < LC_MAX) a.slot[s] = sl;
    s++;
  }
  a.nt = t == s && t <= LC_MAX ? t : -1;
  a.c0 = c0;
  a.c1 = c1;
  a.scale = scale;
  a.twist = twist;
  a.out = out;
  a.out_len = out_len;
  return a;
}

// independent lincombs: one launch when all are 16-byte aligned, else one by one
int lincomb_batch(plk_prover* P, std::initializer_list<LcArgs> list) {
  LcBatch b{};
  int n = 0;
  bool vec = true;
  uint64_t mx = 1;
  for (const LcArgs& a : list) {
    if (a.nt < 0 || n >= LCB_MAX) { plk_set_error("lincomb_batch: bad terms or more than %d", LCB_MAX); return PLK_ERR_ARG; }
    b.a[n++] = a;
    vec = vec && ((uintptr_t)a.out % 16) == 0;
    for (int i = 0; i < a.nt; i++) vec = vec && ((uintptr_t)a.p[i] % 16) == 0;
    mx = std::max<uint64_t>(mx, a.out_len);
  }
  if (!vec) {
    for (int i = 0; i < n; i++) {
      const uint64_t blocks = std::min<uint64_t>((b.a[i].out_len + 255) / 256, 2048);
      hipLaunchKernelGGL(lincomb_kernel, dim3((unsigned)std::max<uint64_t>(blocks, 1)), dim3(256), 0, P->st, b.a[i],
                         P->d_S);
    }
  } else {
    const uint64_t blocks = std::min<uint64_t>((mx + 4095) / 4096, 2048);
    hipLaunchKernelGGL(lincomb16_batch_kernel, dim3((unsigned)std::max<uint64_t>(blocks, 1), n), dim3(256), 0, P->st, b,
                       P->d_S);
  }
  PLK_HIP(hipGetLastError());
  return PLK_OK;
}

int lincomb(plk_prover* P, std::initializer_list<std::pair<const uint8_t*, uint64_t>> terms,
            std::initializer_list<int> slots, int c0, int c1, int scale, int twist, uint8_t* out, uint64_t out_len) {
  LcArgs a{};
  int t = 0;
  for (const auto& pr : terms) { a.p[t] = pr.first; a.len[t] = pr.second; t++; }
  int s = 0;
  for (int sl : slots) a.slot[s++] = sl;
  if (t != s || t > LC_MAX) { plk_set_error("lincomb: %d terms / %d slots", t, s); return PLK_ERR_ARG; }
  a.nt = t;
  a.c0 = c0;
  a.c1 = c1;
  a.scale = scale;
  a.twist = twist;
  a.out = out;
  a.out_len = out_len;
  bool vec = ((uintptr_t)out % 16) == 0;
  for (int i = 0; i < t; i++) vec = vec && ((uintptr_t)a.p[i] % 16) == 0;
  if (vec) {
    const uint64_t blocks = std::min<uint64_t>((out_len + 4095) / 4096, 2048);
    hipLaunchKernelGGL(lincomb16_kernel, dim3((unsigned)std::max<uint64_t>(blocks, 1)), dim3(256), 0, P->st, a,
                       P->d_S);
  } else {
    const uint64_t blocks = std::min<uint64_t>((out_len + 255) / 256, 2048);
    hipLaunchKernelGGL(lincomb_kernel, dim3((unsigned)std::max<uint64_t>(blocks, 1)), dim3(256), 0, P->st, a,
                       P->d_S);
  }
  PLK_HIP(hipGetLastError());
  return PLK_OK;
}

// one evaluation of a batch, or (join) one more row of the previous entry's evaluation
struct EvSpec {
  const uint8_t* p;
  uint64_t len;
  int xslot, out;
  int col = -1;        // chunk-aggregate column (EvArgs::col), -1: none
  int mexp = 0;        // the row's partial enters the evaluation times x^mexp
  bool join = false;   // a further row of the previous entry's evaluation (no split, same out)
};
// agg_ok (optional): false when a row that stores chunk aggregates cannot be read in whole 16-byte
// chunks (the aggregates are then not produced: the caller falls back to the two-launch scan)
EvArgs make_evargs(plk_prover* P, const std::vector<EvSpec>& ev, int post, bool* agg_ok = nullptr, uint8_t* agg = nullptr) {
  EvArgs a{};
  a.agg = agg;
  bool ok = true;
  // a polynomial much longer than the shortest one (t(x): 3n, the r(x) part: 2n) runs as several
  // rows of about the shortest length, so its blocks do no more work than the others' and the
  // launch does not wait on one row's tail
  uint64_t base = ~0ull;
  for (const EvSpec& t : ev) base = std::min<uint64_t>(base, std::max<uint64_t>(t.len, 1));
  int spare = EV_ROWS - (int)ev.size();
  int e = -1, r = 0;
  for (size_t q = 0; q < ev.size(); q++) {
    const EvSpec& t = ev[q];
    const uint8_t* p = t.p;
    const uint64_t len = t.len;
    // 2: aligned and readable in whole 16-byte chunks (length a multiple of 16, or inside the
    // prover's own padded allocation); 1: aligned; 0: bytes
    const bool inside = p >= P->mem && p < P->mem + P->mem_bytes;
    const int vec = ((uintptr_t)p % 16) != 0 ? 0 : ((len % 16 == 0 || inside) ? 2 : 1);
    const int col = agg && vec == 2 ? t.col : -1;
    ok = ok && (t.col < 0 || col >= 0);
    const bool grouped = t.join || (q + 1 < ev.size() && ev[q + 1].join);
    int parts = 1;
    if (!grouped && PLK_EV_SPLIT && vec && base >= 4096 && len >= 2 * base)
      parts = (int)std::min<uint64_t>((len + base / 2) / base, (uint64_t)(1 + spare));
    spare -= parts - 1;
    uint64_t chunk = ((len + parts - 1) / parts + 15) / 16 * 16;
    if (col >= 0) chunk = (chunk + AGG_CHUNK - 1) / AGG_CHUNK * AGG_CHUNK;   // (whole scan chunks per row)
    if (!t.join) e++;
    for (int k = 0; k < parts; k++, r++) {
      const uint64_t off = std::min<uint64_t>(k * chunk, len);
      a.p[r] = p + off;
      a.len[r] = std::min<uint64_t>(chunk, len - off);
      a.xslot[r] = t.xslot;
      a.out[r] = t.out;
      a.vec[r] = vec;   // (off = 0 mod 16: the alignment and the whole-chunk reads carry over)
      a.grp[r] = e;
      a.first[r] = k == 0 && !t.join;
      a.mexp[r] = t.mexp;
      a.col[r] = col;
      a.coff[r] = (int)(off / AGG_CHUNK);
    }
  }
  for (int i = 0; i < r; i++) {   // rows per evaluation: the arrivals its word counts (x blocks)
    a.parts[i] = 0;
    for (int j = 0; j < r; j++) a.parts[i] += a.grp[j] == a.grp[i];
  }
  a.ne = e + 1;
  a.nr = r;
  a.post = post;
  if (agg_ok) *agg_ok = ok && agg;
  return a;
}
EvArgs make_evargs(plk_prover* P, std::initializer_list<std::tuple<const uint8_t*, uint64_t, int, int>> ev, int post) {
  std::vector<EvSpec> v;
  for (const auto& t : ev) v.push_back(EvSpec{std::get<0>(t), std::get<1>(t), std::get<2>(t), std::get<3>(t)});
  return make_evargs(P, v, post);
}
int evals_launch(plk_prover* P, const EvArgs& a, const EarlyMsm* em = nullptr) {
  const int nrows = a.nr;
  EarlyMsm e{};
  if (em && em->nrows > 0) {
    e = *em;
    P->early_rows = e.nrows;
  }
  hipLaunchKernelGGL(eval_kernel, dim3(EV_BLOCKS, nrows + e.nrows), dim3(256), 0, P->st, a, P->d_S, P->d_tick, P->d_stat,
                     e);
  PLK_HIP(hipGetLastError());
  return PLK_OK;
}
int evals(plk_prover* P, std::initializer_list<std::tuple<const uint8_t*, uint64_t, int, int>> ev, int post,
          const EarlyMsm* em = nullptr) {
  const EvArgs a = make_evargs(P, ev, post);
  return evals_launch(P, a, em);
}

int pmul(plk_prover* P, const uint8_t* a, uint64_t la, const uint8_t* b, uint64_t lb, uint8_t* out) {
  return plk_poly_mul_launch(a, la, b, lb, out, nullptr, P->work, P->st);
}

// divide num (upper-bound length nl) by Z_H; q gets ltx bytes
int divide_zh(plk_prover* P, const uint8_t* num, uint64_t nl, uint8_t* q, uint64_t ql, uint32_t* flag) {
  // the binomial kernel writes every q[j < ql] whenever nl > m (one chain per residue)
  if (P->zh_kind != 0 || nl <= P->zh_len - 1) PLK_HIP(hipMemsetAsync(q, 0, ql, P->st));
  P->rem_blocks = 0;
  if (P->zh_kind == 0) {
    const uint64_t m = P->zh_len - 1;
    if (m % 4 == 0 && (uintptr_t)num % 4 == 0 && (uintptr_t)q % 4 == 0 && flag == P->d_stat + ST_REM_T) {
      const uint64_t nb = (m / 4 + 255) / 256;
      hipLaunchKernelGGL(divide_binomial4_kernel, dim3((unsigned)nb), dim3(256), 0, P->st, num, nl, m, P->zh_lead,
                         P->zh_c, q, ql, ql ? (ql - 1) / m : 0, ql ? (ql - 1) % m : 0, P->d_rem);
      P->rem_blocks = nb;   // trim_pack_kernel folds the votes into *flag (ST_REM_T)
    } else {
      hipLaunchKernelGGL(divide_binomial_kernel, dim3((unsigned)((m + 255) / 256)), dim3(256), 0, P->st, num, nl, m,
                         P->zh_lead, P->zh_c, q, ql, flag);
    }
  } else {
    if (nl > (1u << 20)) { plk_set_error("poly_divide: non-binomial Z_H with %llu coefficients", (unsigned long long)nl); return PLK_ERR_RANGE; }
    hipLaunchKernelGGL(divide_general_kernel, dim3(1), dim3(256), 0, P->st, num, nl, P->d_zh, (uint64_t)P->zh_len,
                       P->REMT, q, flag);
  }
  PLK_HIP(hipGetLastError());
  return PLK_OK;
}

// divide num_i by x - S[aslot_i] (i < nd <= 2); q_i gets nl_i - 1 bytes
struct LinDivReq {
  const uint8_t* num;
  uint64_t nl;
  int aslot;
  uint8_t* q;
  uint32_t* flag;
};
// lcs (optional): the numerators' lincombs, computed by the aggregate launch itself
// am (optional, with lcs): the later chunks' aggregates from round 4's evaluation rows -- ONE launch
int divide_linear(plk_prover* P, std::initializer_list<LinDivReq> reqs, const LcBatch* lcs = nullptr,
                  const EarlyMsm* em = nullptr, const AggMap* am = nullptr) {
  if (lcs) {   // a skipped (tiny) division would shift the numerators' order: compute them apart
    int j = 0;
    bool tiny = false;
    for (const LinDivReq& r : reqs) tiny = tiny || r.nl < 2 || lcs->a[j++].out != r.num;
    if (tiny) {
      int rc = PLK_OK;
      for (int i = 0; i < j && !rc; i++) rc = lincomb_batch(P, {lcs->a[i]});
      if (rc) return rc;
      lcs = nullptr;
    }
  }
  LinDivs L{};
  int nd = 0, nbmax = 0;
  uint32_t* bs = P->d_bsum;
  for (const LinDivReq& r : reqs) {
    if (r.nl < 2) {   // quotient [0]; remainder = num (checked by trim)
      PLK_HIP(hipMemsetAsync(r.q, 0, 1, P->st));
      continue;
    }
    const int nb = (int)((r.nl + SCAN_B - 1) / SCAN_B);
    const int vec = ((uintptr_t)r.num % 16 == 0) && ((uintptr_t)r.q % 16 == 0);
    L.d[nd++] = LinDiv{r.num, r.nl, r.aslot, nb, r.q, r.flag, bs, vec};
    bs += nb + 2;
    nbmax = std::max(nbmax, nb);
  }
  if (!nd) return PLK_OK;
  if (lcs && plk_opt(PLK_OPT_PROVE_FUSE_DIV) && (uint32_t)nbmax <= P->scanw_stride) {
    if (++P->scan_epoch == 0) ++P->scan_epoch;   // (words hold 0 after create: never a live epoch)
    hipLaunchKernelGGL(lincomb_divide_kernel, dim3((unsigned)nbmax, nd), dim3(SCAN_T), 0, P->st, *lcs, L, P->d_S,
                       P->d_scanw, P->scanw_stride, P->scan_epoch);
    PLK_HIP(hipGetLastError());
    return PLK_OK;
  }
  if (lcs) {
    EarlyMsm e{};
    e.nd = nd;
    if (em && em->nrows > 0) {
      e = *em;
      e.nd = nd;
      e.X = std::min<uint32_t>(e.X, (uint32_t)nbmax);
      P->early_rows = e.nrows;
    }
    if (am && nd == 2) {   // (both divisions present: the map's rows are [W, ZZ])
      hipLaunchKernelGGL(lincomb_agg_divide_kernel, dim3((unsigned)nbmax, nd + (e.nrows > 0 ? e.nrows : 0)),
                         dim3(AGG_T), 0, P->st, *lcs, L, P->d_S, *am, e);
      PLK_HIP(hipGetLastError());
      return PLK_OK;
    }
    hipLaunchKernelGGL(lincomb_scan_kernel, dim3((unsigned)nbmax, nd + (e.nrows > 0 ? e.nrows : 0)), dim3(SCAN_T), 0,
                       P->st, *lcs, L, P->d_S, e);
  }
  else hipLaunchKernelGGL(lin_scan_sums_kernel, dim3((unsigned)nbmax, nd), dim3(SCAN_T), 0, P->st, L, P->d_S);
  PLK_HIP(hipGetLastError());
  // denominators poly_new({-z, 1}) and ({-z omega, 1}), src/plonk.h:604-613
  hipLaunchKernelGGL(lin_scan_apply_kernel, dim3((unsigned)nbmax, nd), dim3(SCAN_T), 0, P->st, L, P->d_S);
  PLK_HIP(hipGetLastError());
  return PLK_OK;
}

#if PLK_DIAG_DROP_HANDOFF & 1
// diagnostic build only: holds its stream for `ticks` of the 100 MHz wall clock
__global__ void diag_spin_kernel(unsigned long long ticks) {
  const unsigned long long t0 = wall_clock64();
  while (wall_clock64() - t0 < ticks) __builtin_amdgcn_s_sleep(8);
}
#endif

// restores the calling thread's current device on scope exit
struct DevGuard {
  int prev;
  DevGuard() : prev(plk_cur_device()) {}
  ~DevGuard() { (void)hipSetDevice(prev); }
};
// a prover's work runs on ITS device whatever the calling thread's current device is: its stream
// and buffers live there, and the launches look up the NTT / MSM tables by the current device
// (ADVICE r4); the caller's device is restored on return
#define PROVER_ON_DEVICE(P) \
  DevGuard dg_;             \
  PLK_HIP(hipSetDevice((P)->dev))

// plk_prover_create on device `dev` (the library's primary, or a helper's GPU whose tables
// plk_ctx_prepare_device built); the caller's current device is restored
int create_on(const plk_plonk_desc_t* d, int dev, plk_prover_t** out) {
  if (!d || !out) { plk_set_error("plk_prover_create: NULL argument"); return PLK_ERR_ARG; }
  *out = nullptr;
  if (d->n == 0 || !d->z_h || d->z_h_len == 0 || !d->srs_g1 || d->srs_len == 0) {
    plk_set_error("plk_prover_create: n, z_h and srs are required");
    return PLK_ERR_ARG;
  }
  int rc = plk_ctx_retain();
  if (rc) return rc;
  if (dev >= 0 && (rc = plk_ctx_prepare_device(dev))) {
    plk_ctx_release();
    return rc;
  }
  DevGuard dg;
  if (dev >= 0 && hipSetDevice(dev) != hipSuccess) {
    plk_ctx_release();
    plk_set_error("plk_prover_create: hipSetDevice(%d) failed", dev);
    return PLK_ERR_HIP;
  }
  plk_prover* P = new plk_prover();
  P->dev = plk_cur_device();
  P->n = d->n;
  P->srs_len = d->srs_len;
  // Z_H: trimmed as poly_z returns it; classify
  size_t zl = d->z_h_len;
  while (zl > 1 && d->z_h[zl - 1] == 0) zl--;
  if (zl == 1 && d->z_h[0] == 0) {
    delete P;
    plk_ctx_release();
    plk_set_error("Division by zero polynomial in poly_divide");
    return PLK_ERR_ARG;
  }
  P->zh_len = zl;
  P->zh_lead = d->z_h[zl - 1] % HFP;
  P->zh_c = d->z_h[0] % HFP;
  P->zh_kind = 0;
  if (zl < 2) P->zh_kind = 1;
  for (size_t i = 1; i + 1 < zl; i++)
    if (d->z_h[i] % HFP) P->zh_kind = 1;
  P->have_circuit_tables = d->h && d->k1_h && d->k2_h && d->h_pows_inv;

  const Lens L = lens_for(P->n, P->zh_len);
  const uint64_t n = P->n;
  // commitments: a b c z t_lo t_mid t_hi w_z w_zw
  // committed lengths: a b c z (la, lzx), t_lo / t_mid / t_hi (poly_slice of t_x at part = n + 2:
  // <= part, <= part, ltx - 2 part), w_z, w_zw (lwq, lwo) -- t_x itself is never committed
  const uint64_t lthi = L.ltx > 2 * (n + 2) ? L.ltx - 2 * (n + 2) : 1;
  P->cmax = std::max(std::max(L.la, L.lzx), std::max(std::max<uint64_t>(n + 2, lthi), std::max(L.lwq, L.lwo)));
  P->cstride = (P->cmax + 15) & ~(size_t)15;
  // poly_mul workspace: the largest batch of round 3 (rounds()), or a single product
  size_t ws = 0;
  const uint64_t shapes[][2] = {{2, L.lz}, {3, L.lz}, {L.lzx, n}};
  for (const auto& s : shapes) ws = std::max(ws, plk_poly_mul_workspace_bytes(s[0], s[1]));
  const uint64_t g1[][2] = {{L.la, L.la}, {L.la, n}, {L.la, n}, {L.la, n}, {L.la, L.la}, {L.la, L.la}, {L.lz1, n},
                              {L.lzx, n}, {L.la, L.lzx}, {L.la, L.lzw}};
  const uint64_t g2[][2] = {{L.lab, n}, {L.l2a, L.la + L.lzx - 1}, {L.l2a, L.la + L.lzw - 1}};
  size_t w1 = 0, w2 = 0;
  for (const auto& s : g1) w1 += plk_poly_mul_workspace_bytes(s[0], s[1]);
  for (const auto& s : g2) w2 += plk_poly_mul_workspace_bytes(s[0], s[1]);
  ws = std::max(ws, std::max(w1, w2));
  Bump B;
  const size_t o_srs = B.take(3 * P->srs_len + 16), o_zh = B.take(zl + 16), o_h3 = B.take(3 * n + 16),
               o_hinv = B.take(P->have_circuit_tables ? n * n + 16 : 16), o_S = B.take(NSLOT),
               o_stat = B.take(4 * NSTAT), o_tick = B.take(4 * TICK_STRIDE * (EV_MAX + 1)),
               o_rem = B.take(P->zh_len / 1024 + 64),
               o_bsum = B.take(4 * ((L.lw + SCAN_B - 1) / SCAN_B + 2) + 4 * ((L.lzz + SCAN_B) / SCAN_B + 2)),
               o_scanw = B.take(8 * 2 * ((std::max(L.lw, L.lzz) + SCAN_B) / SCAN_B + 2)),
               o_agg = B.take(16 * ((std::max(L.lw, L.lzz) + SCAN_B) / SCAN_B + 2)),
               o_res = B.take(9 * sizeof(PlkMsmResult)),
               o_srslog = B.take(P->srs_len + 16), o_words = B.take(64),
               o_arena = B.take(9 * P->cstride);
  size_t o_polys[13];
  for (int i = 0; i < 13; i++) o_polys[i] = B.take(n + 16);
  const size_t o_cir = B.take(14 * n + 16), o_vals = B.take(11 * n + 16), o_outs = B.take(13 * sizeof(void*));
  struct { uint8_t** p; uint64_t len; } iv[] = {
      {&P->blA, L.lz + 1}, {&P->blB, L.lz + 1}, {&P->blC, L.lz + 1}, {&P->zB, L.lz + 2}, {&P->AB, L.lab},
      {&P->ABQM, L.labqm}, {&P->AQL, L.lq1}, {&P->BQR, L.lq1}, {&P->CQO, L.lq1}, {&P->A2, L.la}, {&P->B2, L.la},
      {&P->C2, L.la}, {&P->T2a, L.l2a}, {&P->T2b, L.l2b}, {&P->T2, L.l2}, {&P->A3, L.la}, {&P->B3, L.la},
      {&P->C3, L.la}, {&P->ZW, L.lzw}, {&P->T3a, L.l2a}, {&P->T3b, L.l2b}, {&P->T3, L.l3}, {&P->Z1, L.lz1},
      {&P->T4, L.lt4}, {&P->NUM, L.lnum}, {&P->TX, L.ltx}, {&P->P3, L.lr3},
      {&P->W, L.lw}, {&P->ZZ, L.lzz}, {&P->REMT, L.lnum}, {&P->ACCV, n}, {&P->E0, n}};
  size_t o_iv[sizeof(iv) / sizeof(iv[0])];
  for (size_t i = 0; i < sizeof(iv) / sizeof(iv[0]); i++) o_iv[i] = B.take(iv[i].len + 16);
  const size_t o_work = B.take(ws + 16);
  P->mem_bytes = B.off;
  if (hipMalloc((void**)&P->mem, P->mem_bytes) != hipSuccess) {
    plk_set_error("plk_prover_create: hipMalloc(%zu) failed", P->mem_bytes);
    delete P;
    plk_ctx_release();
    return PLK_ERR_NOMEM;
  }
  if (hipHostMalloc((void**)&P->h_res, 64 + 4 * NSTAT, hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess ||
      hipHostGetDevicePointer((void**)&P->d_res_host, P->h_res, 0) != hipSuccess) {
    plk_set_error("plk_prover_create: hipHostMalloc of the result buffer failed");
    plk_prover_destroy(P);
    return PLK_ERR_NOMEM;
  }
  memset(P->h_res, 0, 64 + 4 * NSTAT);   // (completion word 0: no call yet)
  uint8_t* m = P->mem;
  P->d_srs = m + o_srs; P->d_zh = m + o_zh; P->d_h3 = m + o_h3; P->d_hinv = m + o_hinv; P->d_S = m + o_S;
  P->d_stat = (uint32_t*)(m + o_stat); P->d_tick = (uint32_t*)(m + o_tick); P->d_rem = m + o_rem; P->d_bsum = (uint32_t*)(m + o_bsum);
  P->d_scanw = (unsigned long long*)(m + o_scanw);
  P->d_agg = m + o_agg;
  P->scanw_stride = (uint32_t)((std::max(L.lw, L.lzz) + SCAN_B) / SCAN_B + 2);
  P->d_res = (PlkMsmResult*)(m + o_res); P->arena = m + o_arena;
  P->d_srs_log = m + o_srslog;
  P->d_srs_flag = (uint32_t*)(m + o_words);
  P->d_done = (uint32_t*)(m + o_words + 4);
  for (int i = 0; i < 13; i++) P->d_polys[i] = m + o_polys[i];
  P->d_cir = m + o_cir; P->d_vals = m + o_vals; P->d_outs = (uint8_t**)(m + o_outs);
  for (size_t i = 0; i < sizeof(iv) / sizeof(iv[0]); i++) *iv[i].p = m + o_iv[i];
  P->work = m + o_work;
  P->work_bytes = ws;
  P->st = nullptr;
  hipError_t e = hipStreamCreateWithFlags(&P->st, hipStreamNonBlocking);
  if (e == hipSuccess) e = hipEventCreateWithFlags(&P->ev, hipEventDisableTiming);
  if (e == hipSuccess) e = hipEventCreateWithFlags(&P->ev_in, hipEventDisableTiming);
  if (e == hipSuccess) e = hipEventCreateWithFlags(&P->ev_done, hipEventDisableTiming);
  if (e == hipSuccess) e = hipMemsetAsync(P->mem, 0, P->mem_bytes, P->st);
  if (e == hipSuccess) e = hipMemcpyAsync(P->d_srs, d->srs_g1, 3 * P->srs_len, hipMemcpyHostToDevice, P->st);
  if (e == hipSuccess) e = hipMemcpyAsync(P->d_zh, d->z_h, zl, hipMemcpyHostToDevice, P->st);
  if (e == hipSuccess && P->have_circuit_tables) {
    e = hipMemcpyAsync(P->d_h3, d->h, n, hipMemcpyHostToDevice, P->st);
    if (e == hipSuccess) e = hipMemcpyAsync(P->d_h3 + n, d->k1_h, n, hipMemcpyHostToDevice, P->st);
    if (e == hipSuccess) e = hipMemcpyAsync(P->d_h3 + 2 * n, d->k2_h, n, hipMemcpyHostToDevice, P->st);
    if (e == hipSuccess) e = hipMemcpyAsync(P->d_hinv, d->h_pows_inv, n * n, hipMemcpyHostToDevice, P->st);
  }
  if (e == hipSuccess) e = hipMemcpyAsync(P->d_outs, P->d_polys, 13 * sizeof(void*), hipMemcpyHostToDevice, P->st);
  if (e != hipSuccess) {
    plk_set_error("plk_prover_create: %s", hipGetErrorString(e));
    plk_prover_destroy(P);
    return PLK_ERR_HIP;
  }
  {  // the SRS in log form, once (the commitments' MSMs read 1 B per point); any non-canonical
     // encoding keeps the G1 form and the exact serial folds
    uint32_t flag = 0;
    P->exp_words = plk_msm_exp_words_dev();
    rc = P->exp_words ? plk_srs_log_launch(P->d_srs, P->srs_len, P->d_srs_log, P->d_srs_flag, P->st) : PLK_ERR_HIP;
    if (!rc && (hipMemcpyAsync(&flag, P->d_srs_flag, 4, hipMemcpyDeviceToHost, P->st) != hipSuccess ||
                hipStreamSynchronize(P->st) != hipSuccess))
      rc = PLK_ERR_HIP;
    if (rc) { plk_prover_destroy(P); return rc; }
    P->srs_irregular = flag != 0;
  }
  *out = P;
  return PLK_OK;
}

void detach_helpers(plk_prover* P);

void drop_graph(plk_prover* P);   // (rounds_graph)
}  // namespace

extern "C" {

int plk_prover_create(const plk_plonk_desc_t* d, plk_prover_t** out) { return create_on(d, -1, out); }

void plk_prover_destroy(plk_prover_t* P) {
  if (!P) return;
  detach_helpers(P);
  DevGuard dg;
  (void)hipSetDevice(P->dev);
  if (P->st) (void)hipStreamSynchronize(P->st);
  drop_graph(P);
  (void)hipFree(P->mem);
  if (P->h_res) (void)hipHostFree(P->h_res);
  (void)hipFree(P->fix_mem);
  (void)hipFree(P->hin);
  for (hipEvent_t e : {P->ev, P->ev_in, P->ev_done, P->tev[0], P->tev[1], P->tev[2], P->tev[3], P->tev[4], P->tev[5]})
    if (e) (void)hipEventDestroy(e);
  if (P->st) (void)hipStreamDestroy(P->st);
  delete P;
  plk_ctx_release();
}

size_t plk_prover_device_bytes(const plk_prover_t* P) { return P ? P->mem_bytes : 0; }

}  // extern "C"

namespace {

// rounds 1-5 (src/plonk.h:277-655) on polys[13] = f_a f_b f_c q_o q_m q_l q_r q_c s1 s2 s3 acc_x l_1_x
// (each of length <= n, zero padded to n).  Enqueued on P->st; status words in P->d_stat.
// Strong-scaled proofs (several GPUs, plk_prover_chains_dev / plk_prover_rounds_ext_dev): the
// round-3 chains t_2 = (A2 B2)(C2 z) and t_3 = (A3 B3)(C3 z(omega x)) depend only on the proof's
// inputs, so another GPU can compute them from the same inputs while this one runs the rest.
struct RoundsMode {
  int ext = 0;                          // chains (PLK_CHAIN_*) whose products come from t2 / t3
  const uint8_t *t2 = nullptr, *t3 = nullptr;
  hipEvent_t ready[2] = {nullptr, nullptr};   // the stream waits for them before reading t2 / t3
  int only = 0;                         // helper: just these chains (into o2 / o3), then return
  uint8_t *o2 = nullptr, *o3 = nullptr;
};

// the 9 commitment rows' MSM lengths: a b c z t_lo t_mid t_hi w_z w_zw (the arena rows' order),
// each its polynomial's upper-bound length (P->cmax's terms), at most the SRS length
MsmRowLens msm_row_lens(const plk_prover* P, const Lens& L) {
  const uint64_t part = L.n + 2, lthi = L.ltx > 2 * part ? L.ltx - 2 * part : 1;
  const uint64_t len[9] = {L.la, L.la, L.la, L.lzx, part, part, lthi, L.lwq, L.lwo};
  MsmRowLens r{};
  for (int i = 0; i < 9; i++)
    r.n[i] = PLK_MSM_ROW_LENS ? std::min<uint64_t>(std::min<uint64_t>(len[i], P->cmax), P->srs_len)
                              : std::min<uint64_t>(P->cmax, P->srs_len);
  return r;
}

// scalar file: challenges, constants and host-derivable powers (src/plonk.h:237-247), and the
// blinding polynomials' coefficients
SlotFile make_slotfile(uint64_t n, const uint8_t chal[5], const uint8_t rnd[9]) {
  SlotFile sf{};
  uint8_t* S = sf.b;
  const uint32_t al = chal[0] % HFP, be = chal[1] % HFP, ga = chal[2] % HFP, z = chal[3] % HFP, v = chal[4] % HFP;
  S[S_ZERO] = 0; S[S_ONE] = 1; S[S_NEG1] = 16;
  S[S_ALPHA] = al; S[S_BETA] = be; S[S_GAMMA] = ga; S[S_Z] = z; S[S_V] = v;
  S[S_OMEGA] = 4; S[S_K1] = 2; S[S_K2] = 3;   // OMEGA_VALUE, K1_VALUE, K2_VALUE (src/plonk.h:12-14)
  S[S_BK1] = be * 2 % HFP; S[S_BK2] = be * 3 % HFP;
  S[S_ALPHA2] = h_pow(al, 2);
  S[S_ZN2] = h_pow(z, n + 2); S[S_Z2N4] = h_pow(z, 2 * n + 4);
  S[S_V2] = h_pow(v, 2); S[S_V3] = h_pow(v, 3); S[S_V4] = h_pow(v, 4); S[S_V5] = h_pow(v, 5); S[S_V6] = h_pow(v, 6);
  S[S_NEGZ] = (uint8_t)((HFP - z) % HFP);
  S[S_ZOMEGA] = (uint8_t)(z * 4 % HFP);
  // blinding polynomials {b2, b1}, {b4, b3}, {b6, b5}, {b9, b8, b7} (src/plonk.h:280-320)
  S[P_BLA] = rnd[1] % HFP; S[P_BLA + 1] = rnd[0] % HFP;
  S[P_BLB] = rnd[3] % HFP; S[P_BLB + 1] = rnd[2] % HFP;
  S[P_BLC] = rnd[5] % HFP; S[P_BLC + 1] = rnd[4] % HFP;
  S[P_BLZ] = rnd[8] % HFP; S[P_BLZ + 1] = rnd[7] % HFP; S[P_BLZ + 2] = rnd[6] % HFP;
  return sf;
}

int rounds(plk_prover* P, const uint8_t* const* pl, const uint8_t chal[5], const uint8_t rnd[9], bool pre = false,
           const RoundsMode& md = RoundsMode{}) {
  const uint64_t n = P->n;
  const Lens L = lens_for(n, P->zh_len);
  const uint8_t *FA = pl[0], *FB = pl[1], *FC = pl[2], *QO = pl[3], *QM = pl[4], *QL = pl[5], *QR = pl[6],
                *QC = pl[7], *S1 = pl[8], *S2 = pl[9], *S3 = pl[10], *ACC = pl[11], *L1 = pl[12];
  const SlotFile sf = make_slotfile(n, chal, rnd);
  // status: stage-A words (gate/copy/acc) are owned by the circuit path; reset the rest
  // (the aligned path's prep_kernel stores the scalar file and clears the status words itself)
  const uint8_t* ins[8] = {P->d_zh, pl[0], pl[1], pl[2], pl[11], pl[8], pl[9], pl[10]};
  bool aligned = true;
  for (const uint8_t* q : ins) aligned = aligned && ((uintptr_t)q % 16) == 0;
  const bool prep = aligned && L.la <= L.lzx && L.lzx <= L.la + 1;
  if (!prep) {
    hipLaunchKernelGGL(scalars_init_kernel, dim3(1), dim3(NSLOT), 0, P->st, sf, P->d_S, P->d_stat, 0, (int)ST_GATE);
    PLK_HIP(hipGetLastError());
  }
  // (the commitment arena needs no clearing: it is zeroed at plk_prover_create and every proof
  // writes the same upper-bound ranges of its 9 slots, so the bytes past them stay zero)
  uint8_t* const cA = P->arena;
  uint8_t* const cB = cA + P->cstride;
  uint8_t* const cC = cB + P->cstride;
  uint8_t* const cZ = cC + P->cstride;
  uint8_t* const cTlo = cZ + P->cstride;
  uint8_t* const cTmid = cTlo + P->cstride;
  uint8_t* const cThi = cTmid + P->cstride;
  uint8_t* const cWz = cThi + P->cstride;
  uint8_t* const cWzw = cWz + P->cstride;
  const uint8_t* dS = P->d_S;
  int rc;
#define RC(x) do { if ((rc = (x))) return rc; } while (0)
  // ---- rounds 1-2 (a_x b_x c_x z_x) and round 3's linear factors, src/plonk.h:280-489
  // Chains: 1 = t_2's (A2 B2, C2 z -> T2), 2 = t_3's (A3 B3, C3 z(omega x) -> T3).  `local`: the
  // chains this call computes itself; a helper call computes only md.only.
  const int local = md.only ? md.only : (PLK_CHAIN_T2 | PLK_CHAIN_T3) & ~md.ext;
  // A2 B2 from a_x b_x when this call computes that product (t2a_kernel after round 3's first
  // batch; a helper computing only the chains keeps the product)
  const bool derive_t2a = (local & PLK_CHAIN_T2) && !md.only && plk_opt(PLK_OPT_PROVE_DERIVE_T2A);
  if (prep) {
    uint8_t* const a2 = (local & PLK_CHAIN_T2) && !derive_t2a ? P->A2 : nullptr;
    uint8_t* const c2 = (local & PLK_CHAIN_T2) ? P->C2 : nullptr;
    uint8_t* const a3 = (local & PLK_CHAIN_T3) ? P->A3 : nullptr;
    const uint64_t blocks = std::min<uint64_t>((L.lzx + 1023) / 1024, 4096);
    const PrepArgs pa{P->d_zh, FA, FB, FC, ACC, S1, S2, S3, L.lz, n, L.la, L.lzx,
                      cA, cB, cC, cZ, a2, P->B2, c2, a3, P->B3, P->C3, P->ZW, P->Z1};
    PLK_MARK(0);
    hipLaunchKernelGGL(prep_kernel, dim3((unsigned)std::max<uint64_t>(blocks, 1)), dim3(256), 0, P->st, pa, sf,
                       P->d_S, P->d_stat, (int)ST_GATE);
    PLK_HIP(hipGetLastError());
    PLK_MARK(1);
  } else {
    // ---- round 1: a_x = (b2 + b1 x) Z_H + f_a, ...  (3 poly_mul)
    RC(pmul(P, dS + P_BLA, 2, P->d_zh, L.lz, P->blA));
    RC(pmul(P, dS + P_BLB, 2, P->d_zh, L.lz, P->blB));
    RC(pmul(P, dS + P_BLC, 2, P->d_zh, L.lz, P->blC));
    RC(lincomb_batch(P, {make_lc({{P->blA, L.lz + 1}, {FA, n}}, {S_ONE, S_ONE}, -1, -1, S_ONE, -1, cA, L.la),
                          make_lc({{P->blB, L.lz + 1}, {FB, n}}, {S_ONE, S_ONE}, -1, -1, S_ONE, -1, cB, L.la),
                          make_lc({{P->blC, L.lz + 1}, {FC, n}}, {S_ONE, S_ONE}, -1, -1, S_ONE, -1, cC, L.la)}));
    // ---- round 2: z_x = (b9 + b8 x + b7 x^2) Z_H + acc_x  (1 poly_mul)
    RC(pmul(P, dS + P_BLZ, 3, P->d_zh, L.lz, P->zB));
    RC(lincomb(P, {{P->zB, L.lz + 2}, {ACC, n}}, {S_ONE, S_ONE}, -1, -1, S_ONE, -1, cZ, L.lzx));
    // ---- round 3: t(x) numerator (12 poly_mul), src/plonk.h:386-503.  The linear factors
    // first, then the products in two batches of independent ones (one launch per NTT pass for
    // a whole batch): 10 at 2n (incl. the 17th and the re-associated C2 z, C3 z(omega x)), 3 at 4n.
    RC(lincomb_batch(P, {
        make_lc({{cA, L.la}}, {S_ONE}, S_GAMMA, S_BETA, S_ALPHA, -1, P->A2, L.la),   // alpha (a + gamma + beta x)
        make_lc({{cB, L.la}}, {S_ONE}, S_GAMMA, S_BK1, S_ONE, -1, P->B2, L.la),      // b + gamma + beta k1 x
        make_lc({{cC, L.la}}, {S_ONE}, S_GAMMA, S_BK2, S_ONE, -1, P->C2, L.la),      // c + gamma + beta k2 x
        make_lc({{cA, L.la}, {S1, n}}, {S_ONE, S_BETA}, S_GAMMA, -1, S_ALPHA, -1, P->A3, L.la),
        make_lc({{cB, L.la}, {S2, n}}, {S_ONE, S_BETA}, S_GAMMA, -1, S_ONE, -1, P->B3, L.la),
        make_lc({{cC, L.la}, {S3, n}}, {S_ONE, S_BETA}, S_GAMMA, -1, S_ONE, -1, P->C3, L.la),
        make_lc({{cZ, L.lzx}}, {S_ONE}, -1, -1, S_ONE, S_OMEGA, P->ZW, L.lzw),       // z(omega x)
        make_lc({{cZ, L.lzx}}, {S_ONE}, S_NEG1, -1, S_ALPHA2, -1, P->Z1, L.lz1)}));  // alpha^2 (z - 1)
  }
  {
    // a_x q_l + b_x q_r + c_x q_o as ONE sum group (one inverse transform) when the sum fits
    // F29's centered range: 3 * 64 n <= (p - 1) / 2 (n <= 1,223,338)
    const int lin = plk_poly_mul_summable(L.la, n) && (uint64_t)3 * L.la * 128 < f29::P ? 1 : 0;
    P->lin_sum = lin;
    // (order: the center launch balances the jobs over its two block halves by pass units,
    // center_schedule; a_x, b_x, z_x are transformed once for their two products each)
    // fixed: the d_polys index of a job's b operand when it is a preprocessed circuit polynomial
    struct J {
      PlkPolyMulJob j;
      int fixed;
    };
    std::vector<J> g1, g2;
    if (!md.only) {
      g1.push_back({{cA, L.la, QL, n, P->AQL}, 5});
      g1.push_back({{cB, L.la, QR, n, P->BQR, lin}, 6});
      g1.push_back({{cC, L.la, QO, n, P->CQO, lin}, 3});
      g1.push_back({{P->Z1, L.lz1, L1, n, P->T4}, 12});
      g1.push_back({{cA, L.la, cB, L.la, P->AB}, -1});
      // the 17th poly_mul, z_x s_sigma_3 (src/plonk.h:560), as z_x * s3: its scalar beta
      // z_omega_z (a round-4 value) moves into r(x)'s lincomb (S_R3B), so the product joins this batch
      g1.push_back({{cZ, L.lzx, S3, n, P->P3}, 10});
    }
    // t_2 = ((A2 B2) C2) z and t_3 = ((A3 B3) C3) z(omega x) (src/plonk.h:432-434, 471-473)
    // re-associated as (A2 B2)(C2 z): C2 z and C3 z(omega x) join this batch and the 4n products
    // come in one batch (associativity over GF(17); the centered F29 residues hold the 2n x 2n
    // products exactly)
    if (local & PLK_CHAIN_T2) {
      if (!derive_t2a) g1.push_back({{P->A2, L.la, P->B2, L.la, P->T2a}, -1});
      g1.push_back({{P->C2, L.la, cZ, L.lzx, P->T2b}, -1});
    }
    if (local & PLK_CHAIN_T3) {
      g1.push_back({{P->A3, L.la, P->B3, L.la, P->T3a}, -1});
      g1.push_back({{P->C3, L.la, P->ZW, L.lzw, P->T3b}, -1});
    }
    // (a b) q_m ADDED into t_2 = (A2 B2)(C2 z) when both run here and their sum fits F29's
    // centered range, 64 (min(l2a, la + lzx - 1) + min(lab, n)) <= (p - 1) / 2 (n <= ~1.2 M): one
    // 4n inverse transform fewer, one numerator term fewer (t_3 enters with -1, so it stays apart).
    // A group runs in ONE transform size: t_2 has 4n + 6 coefficients and (a b) q_m 3n + 2, so for
    // many n (2100, 5000, 600000, ...) the two plans differ and (a b) q_m stays its own job.
    const uint64_t t2b = L.la + L.lzx - 1;
    const int grp = !md.only && (local & PLK_CHAIN_T2) && plk_poly_mul_summable(L.lab, n) &&
                            plk_poly_mul_summable(L.l2a, t2b) &&
                            plk_poly_mul_transform_plan(L.lab, n, nullptr) ==
                                plk_poly_mul_transform_plan(L.l2a, t2b, nullptr) &&
                            (std::min(L.l2a, t2b) + std::min<uint64_t>(L.lab, n)) * 128 < f29::P
                        ? 1
                        : 0;
    P->t2_sum = grp;
    if (local & PLK_CHAIN_T2) g2.push_back({{P->T2a, L.l2a, P->T2b, t2b, md.only ? md.o2 : P->T2}, -1});
    // PLK_OPT_PROVE_DERIVE_T2A 2: A2 B2's bytes computed by the t_2 product's first forward pass
    // (which stores them to T2a as well) instead of t2a_kernel -- one launch fewer; products on
    // 2^13 tiles only (2^21 and up by default, PLK_OPT_NTT_T13_MIN_K), else t2a_kernel
    const WDerive dv{P->AB, cA, cB, dS, L.la, L.lab, S_ALPHA, S_BETA, S_GAMMA, S_BK1};
    const bool derive_fwd = derive_t2a && plk_opt(PLK_OPT_PROVE_DERIVE_T2A) == 2 && L.l2a == L.lab &&
                            plk_poly_mul_transform_plan(L.l2a, t2b, nullptr) >=
                                std::max<int64_t>(14, plk_opt(PLK_OPT_NTT_T13_MIN_K));
    if (derive_fwd) g2.back().j.der = &dv;
    if (!md.only) g2.push_back({{P->AB, L.lab, QM, n, P->ABQM, grp}, 4});
    if (local & PLK_CHAIN_T3) g2.push_back({{P->T3a, L.l2a, P->T3b, L.la + L.lzw - 1, md.only ? md.o3 : P->T3}, -1});
    if (pre) {   // preprocessed circuit: the fixed b operands' transforms (plk_prover_preprocess)
      for (auto* g : {&g1, &g2})
        for (J& x : *g) {
          if (x.fixed < 0) continue;
          const plk_prover::Fixed& f = P->fix[x.fixed];
          if (f.t && f.src == pl[x.fixed] && x.j.b == pl[x.fixed]) {
            x.j.bt = f.t;
            x.j.bt_k = f.k;
            x.j.bt_field = f.field;
          }
        }
    }
    for (auto* g : {&g1, &g2}) {
      std::vector<PlkPolyMulJob> jobs;
      for (const J& x : *g) jobs.push_back(x.j);
      const int te = g == &g1 ? 1 : 3;   // (plk_prover_profile_dev)
      if (P->tev_on) PLK_HIP(hipEventRecord(P->tev[te], P->st));
      if (!jobs.empty()) RC(plk_poly_mul_batch_launch(jobs.data(), (int)jobs.size(), P->work, P->work_bytes, P->st));
      if (P->tev_on) PLK_HIP(hipEventRecord(P->tev[te + 1], P->st));
      if (g == &g1 && derive_t2a && !derive_fwd) {   // (a_x b_x is complete on the stream here)
        const uint64_t blocks = std::min<uint64_t>((L.lab + 1023) / 1024, 4096);
        hipLaunchKernelGGL(t2a_kernel, dim3((unsigned)std::max<uint64_t>(blocks, 1)), dim3(256), 0, P->st, P->AB, cA, cB,
                           L.la, L.lab, dS, P->T2a);
        PLK_HIP(hipGetLastError());
      }
    }
    if (md.only) return PLK_OK;   // helper: the chains' products are enqueued
  }
  const uint8_t* const T2 = (md.ext & PLK_CHAIN_T2) ? md.t2 : P->T2;
  const uint8_t* const T3 = (md.ext & PLK_CHAIN_T3) ? md.t3 : P->T3;
  for (hipEvent_t e : md.ready)   // their bytes have arrived (the only wait of a split proof)
    if (md.ext && e) PLK_HIP(hipStreamWaitEvent(P->st, e, 0));
  // t(x) = numerator / Z_H; t_lo / t_mid / t_hi = poly_slice(t_x, ...) with part n + 2
  // (src/plonk.h:494-519)
  const uint64_t part = n + 2;
  const uint64_t lmid = L.ltx > part ? std::min<uint64_t>(part, L.ltx - part) : 0;
  const uint64_t lhi = L.ltx > 2 * part ? L.ltx - 2 * part : 0;
  // (the sums in AQL / T2 stand for their members' terms)
  LcArgs num = P->lin_sum
                   ? make_lc({{P->ABQM, L.labqm}, {P->AQL, L.lq1}, {QC, n}, {T2, L.l2}, {T3, L.l3}, {P->T4, L.lt4}},
                             {S_ONE, S_ONE, S_ONE, S_ONE, S_NEG1, S_ONE}, -1, -1, S_ONE, -1, P->NUM, L.lnum)
                   : make_lc({{P->ABQM, L.labqm}, {P->AQL, L.lq1}, {P->BQR, L.lq1}, {P->CQO, L.lq1}, {QC, n},
                              {T2, L.l2}, {T3, L.l3}, {P->T4, L.lt4}},
                             {S_ONE, S_ONE, S_ONE, S_ONE, S_ONE, S_ONE, S_NEG1, S_ONE}, -1, -1, S_ONE, -1, P->NUM,
                             L.lnum);
  if (P->t2_sum) {   // drop the ABQM term (first)
    for (int t = 1; t < num.nt; t++) {
      num.p[t - 1] = num.p[t];
      num.len[t - 1] = num.len[t];
      num.slot[t - 1] = num.slot[t];
    }
    num.nt--;
  }
  // (q_c is the caller's buffer: n % 4 == 0 keeps its last dword inside it; the intermediates
  // carry >= 16 bytes of padding)
  bool fused = P->zh_kind == 0 && (P->zh_len - 1) % 4 == 0 && L.lnum > P->zh_len - 1 && num.nt >= 5 && num.nt <= 8 &&
               (uintptr_t)P->TX % 4 == 0 && n % 4 == 0 && (P->zh_len - 1) / 4 < (1ull << 31) && L.ltx / (P->zh_len - 1) < 8;
  for (int t = 0; t < num.nt; t++) fused = fused && (uintptr_t)num.p[t] % 4 == 0;
  if (fused) {
    const uint64_t m = P->zh_len - 1, ql = L.ltx, nb = (m / 4 + 255) / 256;
    const Slices3 sl{{cTlo, cTmid, cThi}, {std::min<uint64_t>(part, L.ltx), lmid, lhi}, part};
    const uint64_t cq = ql ? (ql - 1) / m : 0, cr = ql ? (ql - 1) % m : 0;
#define PLK_NUMDIV(NT_, K_)                                                                                      \
  hipLaunchKernelGGL((numdiv_kernel<NT_, K_>), dim3((unsigned)nb), dim3(256), 0, P->st, num, dS, m, P->zh_lead, P->zh_c, \
                     P->TX, ql, cq, cr, sl, P->d_rem)
    // (5..8 terms: with / without the two sums)
    const bool k4 = cq + 1 <= 4;
    switch (num.nt) {
      case 5: if (k4) PLK_NUMDIV(5, 4); else PLK_NUMDIV(5, 8); break;
      case 6: if (k4) PLK_NUMDIV(6, 4); else PLK_NUMDIV(6, 8); break;
      case 7: if (k4) PLK_NUMDIV(7, 4); else PLK_NUMDIV(7, 8); break;
      default: if (k4) PLK_NUMDIV(8, 4); else PLK_NUMDIV(8, 8); break;
    }
#undef PLK_NUMDIV
    PLK_HIP(hipGetLastError());
    P->rem_blocks = nb;   // trim_pack_kernel folds the votes into ST_REM_T
  } else {
    RC(lincomb_batch(P, {num}));
    RC(divide_zh(P, P->NUM, L.lnum, P->TX, L.ltx, P->d_stat + ST_REM_T));
    const Copy3 c{{P->TX, P->TX + part, P->TX + 2 * part}, {cTlo, cTmid, cThi},
                  {std::min<uint64_t>(part, L.ltx), lmid, lhi}};
    const uint64_t blocks = std::min<uint64_t>((c.len[0] + 255) / 256, 2048);
    hipLaunchKernelGGL(copy3_kernel, dim3((unsigned)std::max<uint64_t>(blocks, 1), 3), dim3(256), 0, P->st, c);
    PLK_HIP(hipGetLastError());
  }
  // ---- round 4: evaluations at z (src/plonk.h:527-533) and r(x)
  // r(x) = ab q_m + a_z q_l + b_z q_r + c_z q_o + (r2 + r4) z_x + r3 z_x (s_sigma_3 beta z_omega_z)
  // (src/plonk.h:536-571; the last product is z_x s_sigma_3 from round 3 times r3 beta z_omega_z).
  // r(x) is never materialised: r_z comes from its terms' evaluations (scalars_r4) and w_z(x)
  // takes v r(x) term by term.  One launch: the 14 evaluations + rounds 4/5 scalar programs.
  // the 7 commitments that do not wait for round 5 (a b c z t_lo t_mid t_hi) as extra grid rows of
  // this launch (PLK_OPT_PROVE_EARLY_COMMITS = 2) or of round 5's scan launch (= 1); log-form SRS
  // and the fused packing only -- commit_pack_kernel then runs w_z, w_z_omega and packs
  P->early_rows = 0;
  const int64_t early = !P->srs_irregular && plk_opt(PLK_OPT_PROVE_SRS_LOGS) && plk_opt(PLK_OPT_PROVE_PACK_FUSE)
                            ? plk_opt(PLK_OPT_PROVE_EARLY_COMMITS)
                            : 0;
  const MsmRowLens rl = msm_row_lens(P, L);
  const EarlyMsm em{P->d_srs_log, P->arena, (uint64_t)P->cstride, rl, P->d_res, P->exp_words, 7, 0, (uint32_t)(2048 / 9)};
  // round 5's numerators (built here: with PLK_OPT_PROVE_EVAL_AGG round 4's evaluation rows also
  // store their terms' scan-chunk aggregates, lincomb_agg_divide_kernel)
  LcBatch nb5{};
  // w_z(x)'s numerator terms, in agg column order (column t = term t): t_lo t_mid t_hi q_m q_l q_r
  // q_o z_x P3 a_x b_x c_x s_sigma_1 s_sigma_2; column 14 = z(omega x) at z = z_x at z omega
  enum { AC_TLO, AC_TMID, AC_THI, AC_QM, AC_QL, AC_QR, AC_QO, AC_ZX, AC_P3, AC_A, AC_B, AC_C, AC_S1, AC_S2, AC_ZW };
  nb5.a[0] = make_lc({{cTlo, std::min<uint64_t>(part, L.ltx)}, {cTmid, lmid}, {cThi, lhi}, {QM, n}, {QL, n},
                      {QR, n}, {QO, n}, {cZ, L.lzx}, {P->P3, L.lr3}, {cA, L.la}, {cB, L.la}, {cC, L.la}, {S1, n},
                      {S2, n}},
                     {S_ONE, S_ZN2, S_Z2N4, S_VAB, S_VAZ, S_VBZ, S_VCZ, S_VR24, S_VR3B, S_V2, S_V3, S_V4, S_V5,
                      S_V6},
                     S_W0, -1, S_ONE, -1, P->W, L.lw);
  nb5.a[1] = make_lc({{cZ, L.lzx}}, {S_ONE}, S_NEGZWZ, -1, S_ONE, -1, P->ZZ, L.lzz);
  // fused numerators need 16-byte aligned terms readable in whole 16-byte chunks: the
  // caller's polynomials (length n) qualify when n % 16 == 0 and they are aligned
  bool fuse = n % 16 == 0 && nb5.a[0].nt > 0 && nb5.a[1].nt > 0;
  for (int j = 0; j < 2; j++) {
    fuse = fuse && (uintptr_t)nb5.a[j].out % 16 == 0;
    for (int t = 0; t < nb5.a[j].nt; t++) fuse = fuse && (uintptr_t)nb5.a[j].p[t] % 16 == 0;
  }
  bool agg = fuse && P->d_agg && plk_opt(PLK_OPT_PROVE_EVAL_AGG) && !plk_opt(PLK_OPT_PROVE_FUSE_DIV) &&
             L.lw >= 2 && L.lzz >= 2;
  EvArgs ea{};
  if (agg) {   // t(z) from its three slices (x^(n + 2), x^(2n + 4): their offsets), every W term's chunks
    const int m1 = (int)(part % 16), m2 = (int)(2 * part % 16);
    ea = make_evargs(P,
                     {{cA, L.la, S_Z, S_AZ, AC_A}, {cB, L.la, S_Z, S_BZ, AC_B}, {cC, L.la, S_Z, S_CZ, AC_C},
                      {S1, n, S_Z, S_S1Z, AC_S1}, {S2, n, S_Z, S_S2Z, AC_S2},
                      {cTlo, std::min<uint64_t>(part, L.ltx), S_Z, S_TZ, AC_TLO},
                      {cTmid, lmid, S_Z, S_TZ, AC_TMID, m1, true}, {cThi, lhi, S_Z, S_TZ, AC_THI, m2, true},
                      {P->ZW, L.lzw, S_Z, S_ZWZ, AC_ZW}, {L1, n, S_Z, S_L1Z},
                      {QM, n, S_Z, S_QMZ, AC_QM}, {QL, n, S_Z, S_QLZ, AC_QL}, {QR, n, S_Z, S_QRZ, AC_QR},
                      {QO, n, S_Z, S_QOZ, AC_QO}, {cZ, L.lzx, S_Z, S_ZXZ, AC_ZX}, {P->P3, L.lr3, S_Z, S_P3Z, AC_P3}},
                     EV_POST_R4, &agg, P->d_agg);
  }
  if (!agg)
    ea = make_evargs(P, {{cA, L.la, S_Z, S_AZ}, {cB, L.la, S_Z, S_BZ}, {cC, L.la, S_Z, S_CZ}, {S1, n, S_Z, S_S1Z},
                         {S2, n, S_Z, S_S2Z}, {P->TX, L.ltx, S_Z, S_TZ}, {P->ZW, L.lzw, S_Z, S_ZWZ}, {L1, n, S_Z, S_L1Z},
                         {QM, n, S_Z, S_QMZ}, {QL, n, S_Z, S_QLZ}, {QR, n, S_Z, S_QRZ}, {QO, n, S_Z, S_QOZ},
                         {cZ, L.lzx, S_Z, S_ZXZ}, {P->P3, L.lr3, S_Z, S_P3Z}},
                     EV_POST_R4);
  RC(evals_launch(P, ea, early == 2 ? &em : nullptr));
  // ---- round 5: opening polynomials (src/plonk.h:580-621)
  // w_z numerator and z(x) - z_omega_z, then both divisions: one launch with the aggregates of
  // round 4, else each pair in one launch per phase
  {
    AggMap am{};
    if (agg) {
      am.agg = P->d_agg;
      for (int t = 0; t < LC_MAX; t++) am.col[0][t] = am.col[1][t] = -1;
      for (int t = 0; t < nb5.a[0].nt; t++) am.col[0][t] = (int8_t)t;   // (AC_* order)
      am.col[1][0] = AC_ZW;
    }
    if (!fuse) RC(lincomb_batch(P, {nb5.a[0], nb5.a[1]}));
    RC(divide_linear(P, {{P->W, L.lw, S_Z, cWz, P->d_stat + ST_REM_W1},
                         {P->ZZ, L.lzz, S_ZOMEGA, cWzw, P->d_stat + ST_REM_W2}},
                     fuse ? &nb5 : nullptr, early == 1 ? &em : nullptr, agg ? &am : nullptr));
  }
  // ---- trimmed lengths for the reference's exits: computed by the packing kernel after the MSM
  TrimArgs trims{};
  int ntrims = 0;
  {
    TrimArgs t{};
    const uint8_t* cps[9] = {cA, cB, cC, cZ, cTlo, cTmid, cThi, cWz, cWzw};
    const uint64_t ub[9] = {L.la, L.la, L.la, L.lzx, std::min<uint64_t>(part, L.ltx), lmid, lhi, L.lwq, L.lwo};
    for (int i = 0; i < 9; i++) { t.p[i] = cps[i]; t.len[i] = std::max<uint64_t>(ub[i], 1); t.dst[i] = ST_LEN0 + i; }
    t.p[9] = P->TX; t.len[9] = L.ltx; t.dst[9] = ST_TXLEN;
    int nt = 10;
    if (P->rem_blocks) { t.p[10] = P->d_rem; t.len[10] = P->rem_blocks; t.dst[10] = ST_REM_T | TRIM_ANY; nt = 11; }
    trims = t;
    ntrims = nt;
  }
  // ---- the 9 commitments: one batched MSM over the arena (srs_eval_at_s, src/srs.h:53-68)
  const uint64_t nm = std::min<uint64_t>(P->cmax, P->srs_len);
  // (the 9 result records are zeroed at plk_prover_create and every launch leaves them re-armed)
  if (!P->srs_irregular && plk_opt(PLK_OPT_PROVE_SRS_LOGS) && plk_opt(PLK_OPT_PROVE_PACK_FUSE)) {
    // commitments + trimmed lengths + packing in one launch (commit_pack_kernel)
    const int row0 = P->early_rows == 7 ? 7 : 0, nrows = 9 - row0;
    // (blocks per row: one 16-point group per thread up to PLK_CP_BX blocks)
    const uint64_t bx = std::max<uint64_t>(std::min<uint64_t>(PLK_CP_BX, std::max<uint64_t>(1, ((nm >> 4) + CP_T - 1) / CP_T)),
                                           (uint64_t)ntrims);
    hipLaunchKernelGGL(commit_pack_kernel, dim3((unsigned)bx, nrows + 1), dim3(CP_T), 0, P->st, P->d_srs_log, P->arena,
                       (uint64_t)P->cstride, msm_row_lens(P, L), P->d_res, P->exp_words, row0, nrows, trims, ntrims, P->d_S, P->d_stat,
                       P->d_res_host, ++P->seq, P->d_done);
    PLK_HIP(hipGetLastError());
    PLK_MARK(7);
    if (PLK_HOST_MARKS) plk_host_marks_print();
    return PLK_OK;
  }
  if (!P->srs_irregular && plk_opt(PLK_OPT_PROVE_SRS_LOGS)) {
    RC(plk_msm_log_batch_launch(P->d_srs_log, 0, P->arena, P->cstride, nm, 9, P->d_res, P->st));
  } else if (!P->srs_irregular) {
    RC(plk_msm_batch_launch(P->d_srs, 0, P->arena, P->cstride, nm, 9, P->d_res, P->st));
  } else {
    for (int i = 0; i < 9; i++) RC(plk_msm_serial_launch(P->d_srs, P->arena + i * P->cstride, nm, P->d_res + i, P->st));
  }
  // (each record's finishing block already wrote its point: no finalize launch)
  hipLaunchKernelGGL(trim_pack_kernel, dim3(1), dim3(PACK_T), 0, P->st, trims, ntrims, P->d_res, P->d_S, P->d_stat,
                     P->d_res_host, ++P->seq);
  PLK_HIP(hipGetLastError());
#undef RC
  return PLK_OK;
}

// the reference's exits, in the order plonk_prove would hit them
int check_status(const plk_prover* P, const uint32_t* st, int strict, int circuit) {
  const uint64_t part = P->n + 2;
  if (circuit && st[ST_GATE]) { plk_set_error("Constraint %u not satisfied.", st[ST_GATE] - 1); return PLK_ERR_ARG; }
  if (circuit && st[ST_COPY]) { plk_set_error("Invalid copy_of type"); return PLK_ERR_ARG; }
  for (int i = 0; i < 3; i++)
    if (st[ST_LEN0 + i] > P->srs_len) { plk_set_error("SRS length is less than polynomial length"); return PLK_ERR_RANGE; }
  if (circuit && strict && st[ST_ACC] != 1) { plk_set_error("assertion acc_x(omega^n) == 1 failed"); return PLK_ERR_ARG; }
  if (st[ST_LEN0 + 3] > P->srs_len) { plk_set_error("SRS length is less than polynomial length"); return PLK_ERR_RANGE; }
  if (strict && st[ST_REM_T]) { plk_set_error("Non-zero remainder in t(x) division"); return PLK_ERR_ARG; }
  if (st[ST_TXLEN] <= 2 * part) { plk_set_error("Invalid slice indices in poly_slice"); return PLK_ERR_RANGE; }
  for (int i = 4; i < 7; i++)
    if (st[ST_LEN0 + i] > P->srs_len) { plk_set_error("SRS length is less than polynomial length"); return PLK_ERR_RANGE; }
  if ((st[ST_REM_W1] | st[ST_REM_W2]) & SCAN_TIMEOUT) {   // (lincomb_divide_kernel: a wait gave up)
    plk_set_error("internal: round-5 division scan timed out waiting for a chunk aggregate");
    return PLK_ERR_HIP;
  }
  if (strict && st[ST_REM_W1]) { plk_set_error("assertion poly_is_zero(&rem1) failed"); return PLK_ERR_ARG; }
  if (strict && st[ST_REM_W2]) { plk_set_error("assertion poly_is_zero(&rem2) failed"); return PLK_ERR_ARG; }
  for (int i = 7; i < 9; i++)
    if (st[ST_LEN0 + i] > P->srs_len) { plk_set_error("SRS length is less than polynomial length"); return PLK_ERR_RANGE; }
  return PLK_OK;
}

int finish(plk_prover* P, int strict, int circuit, uint8_t proof[34]) {
  // trim_pack_kernel wrote P->h_res (mapped pinned) and then this call's completion word: poll it
  // (the stream's own completion is noticed later than the word; PLK_OPT_PROVE_SYNC = 1 waits for
  // the stream instead).  A failed launch never writes it: the stream is queried now and then.
  // Each poll is followed by a pause, and after ~1 ms of polling by a yield, so a waiting prover
  // does not starve the other host threads of a core.
  bool seen = false;
  if (!plk_opt(PLK_OPT_PROVE_SYNC)) {
    const uint32_t* w = (const uint32_t*)(P->h_res + 60);
    for (uint64_t it = 1;; it++) {
      if (__atomic_load_n(w, __ATOMIC_ACQUIRE) == P->seq) { seen = true; break; }
      if (!(it & 4095) && hipStreamQuery(P->st) != hipErrorNotReady) break;   // done (word re-read below) or failed
      __builtin_ia32_pause();
      if (it > 16384) sched_yield();
    }
  }
  if (!seen) {
    PLK_HIP(hipStreamSynchronize(P->st));
    if (__atomic_load_n((const uint32_t*)(P->h_res + 60), __ATOMIC_ACQUIRE) != P->seq) {
      plk_set_error("prover: the packing kernel did not complete");
      return PLK_ERR_HIP;
    }
  }
  uint32_t hs[NSTAT];
  memcpy(hs, P->h_res + 64, sizeof hs);
  const int rc = check_status(P, hs, strict, circuit);
  if (rc) return rc;
  if (proof) memcpy(proof, P->h_res, 34);
  return PLK_OK;
}

// ---- one proof over several GPUs from C (plk_prover_attach_helpers)
// the d_polys entries a helper's chains read: f_a f_b f_c s_sigma_1..3 acc_x (rounds(): prep_kernel
// or its fallback; md.only returns before anything else is read)
constexpr int HELPER_IN[7] = {0, 1, 2, 8, 9, 10, 11};

size_t hin_stride(uint64_t n) { return (n + 16 + 255) & ~(size_t)255; }

void detach_helpers(plk_prover* P) {
  for (int h = 0; h < P->nhelp; h++) {
    plk_prover_destroy(P->help[h]);
    P->help[h] = nullptr;
    P->help_mask[h] = 0;
  }
  P->nhelp = 0;
  if (P->rx_mem) {
    DevGuard dg;
    (void)hipSetDevice(P->dev);
    (void)hipStreamSynchronize(P->st);
    (void)hipFree(P->rx_mem);
  }
  P->rx_mem = nullptr;
  P->rx[0] = P->rx[1] = nullptr;
}

// Rounds 1-5 with the helpers' chains.  Ordering: P->st records ev_in after
// everything already enqueued on it (a circuit's stage A; nothing for device-resident inputs);
// each helper's stream waits for ev_in, copies the 7 inputs it reads to its own device when it
// is another GPU (hipMemcpyPeerAsync), runs its chains, copies the products into P->rx on the
// proving device (hipMemcpyPeerAsync on the helper's stream) and records ev_done; P's stream
// runs everything else and waits for the ev_done events only before the numerator.
int rounds_split(plk_prover* P, const uint8_t* const* pl, const uint8_t* const* hpl, const uint8_t chal[5],
                 const uint8_t rnd[9], bool pre) {
  DevGuard dg;
  PLK_HIP(hipSetDevice(P->dev));
  PLK_HIP(hipEventRecord(P->ev_in, P->st));
  const Lens L = lens_for(P->n, P->zh_len);
  const uint64_t clen[2] = {L.l2 + 16, L.l3 + 16};   // (the numerator reads whole dwords, masked)
  RoundsMode md;
  int rc = PLK_OK;
  for (int h = 0; h < P->nhelp && !rc; h++) {
    plk_prover* H = P->help[h];
    if (hipSetDevice(H->dev) != hipSuccess || hipStreamWaitEvent(H->st, P->ev_in, 0) != hipSuccess) {
      plk_set_error("split proof: helper %d (device %d) cannot wait for the inputs", h, H->dev);
      rc = PLK_ERR_HIP;
      break;
    }
    const uint8_t* hp[13];
    for (int i = 0; i < 13; i++) hp[i] = hpl ? hpl[13 * (h + 1) + i] : pl[i];
    // another GPU (or PLK_OPT_PROVE_HELPER_COPY, which runs this branch on the proving device so
    // that a one-GPU box executes it): the 7 inputs the chains read are copied to the helper's
    // buffers, and the 6 it must not read point at the helper's poison row (0x05 bytes, set at
    // attach) -- never at the proving GPU's memory; a read of one changes the proof
    if (!hpl && (H->dev != P->dev || plk_opt(PLK_OPT_PROVE_HELPER_COPY))) {
      const size_t st = hin_stride(P->n);
      for (int i = 0; i < 13; i++) hp[i] = H->hin + 7 * st;
      for (int q = 0; q < 7 && !rc; q++) {
        uint8_t* dst = H->hin + q * st;
        hp[HELPER_IN[q]] = dst;
#if PLK_DIAG_DROP_HANDOFF & 4   // diagnostic build only (tests/test_prove_helpers_gpu.py): f_a not copied
        if (q == 0) continue;
#endif
        if (hipMemcpyPeerAsync(dst, H->dev, pl[HELPER_IN[q]], P->dev, P->n, H->st) != hipSuccess) {
          plk_set_error("split proof: input copy to device %d failed", H->dev);
          rc = PLK_ERR_HIP;
        }
      }
      if (rc) break;
    }
    RoundsMode hm;
    hm.only = P->help_mask[h];
    hm.o2 = H->T2;
    hm.o3 = H->T3;
    if ((rc = rounds(H, hp, chal, rnd, false, hm))) break;
    for (int c = 0; c < 2 && !rc; c++) {
      if (!(hm.only & (1 << c))) continue;
      const uint8_t* src = c ? H->T3 : H->T2;
      const hipError_t e = H->dev == P->dev
                               ? hipMemcpyAsync(P->rx[c], src, clen[c], hipMemcpyDeviceToDevice, H->st)
                               : hipMemcpyPeerAsync(P->rx[c], P->dev, src, H->dev, clen[c], H->st);
      if (e != hipSuccess) {
        plk_set_error("split proof: product copy from device %d failed: %s", H->dev, hipGetErrorString(e));
        rc = PLK_ERR_HIP;
      }
    }
    if (!rc && hipEventRecord(H->ev_done, H->st) != hipSuccess) rc = PLK_ERR_HIP;
    md.ready[h] = H->ev_done;
    md.ext |= hm.only;
  }
  if (rc) {
    for (int h = 0; h < P->nhelp; h++) {
      (void)hipSetDevice(P->help[h]->dev);
      (void)hipStreamSynchronize(P->help[h]->st);
    }
    return rc;
  }
  PLK_HIP(hipSetDevice(P->dev));
  md.t2 = P->rx[0];
  md.t3 = P->rx[1];
  return rounds(P, pl, chal, rnd, pre, md);
}

// ---- rounds() as a HIP graph (PLK_OPT_PROVE_GRAPH).  A proof is 12-14 dependent launches whose
// host cost (~3-7 us each under a runtime trace) exceeds the GPU time of the first kernels: the GPU
// idles after the first one until the host has enqueued the next.  rounds() enqueues the same
// launches with the same arguments for the same input addresses, options and preprocessed state
// -- except the scalar file (the first kernel's argument: prep_kernel or scalars_init_kernel) and
// the completion word (the last: commit_pack_kernel or trim_pack_kernel) -- so it is captured once
// and replayed: the scalar file set as a node parameter when it changed, the completion word
// cleared by the host before the launch (the call is synchronous: the previous replay is done)
// and polled for the captured value.
void drop_graph(plk_prover* P) {
  if (P->gx) (void)hipGraphExecDestroy(P->gx);
  if (P->g) (void)hipGraphDestroy(P->g);
  P->gx = nullptr;
  P->g = nullptr;
  P->g_first = P->g_last = nullptr;
}

bool graph_matches(const plk_prover* P, const uint8_t* const* pl, bool pre) {
  if (!P->gx || P->g_pre != pre || P->g_fix_gen != P->fix_gen) return false;
  for (int i = 0; i < 13; i++)
    if (P->g_pl[i] != pl[i]) return false;
  for (int o = 1; o < PLK_OPT_COUNT; o++)
    if (P->g_opt[o] != plk_opt(o)) return false;
  return true;
}

// argument idx (of nargs) of kernel node `node` set to *val in the executable graph
int graph_set_arg(plk_prover* P, hipGraphNode_t node, int nargs, int idx, void* val) {
  hipKernelNodeParams kp{};
  PLK_HIP(hipGraphKernelNodeGetParams(node, &kp));
  if (!kp.kernelParams || nargs > 16) {
    plk_set_error("prover graph: kernel node without argument pointers");
    return PLK_ERR_HIP;
  }
  void* args[16];
  for (int i = 0; i < nargs; i++) args[i] = kp.kernelParams[i];
  args[idx] = val;
  kp.kernelParams = args;
  PLK_HIP(hipGraphExecKernelNodeSetParams(P->gx, node, &kp));
  return PLK_OK;
}

// rounds() through the graph: capture (and launch) on a key change, else set the two per-call
// parameters and replay.  The fused division's scan epochs (PLK_OPT_PROVE_FUSE_DIV) change per
// call inside its launch: that mode runs rounds() directly.
int rounds_graph(plk_prover* P, const uint8_t* const* pl, const uint8_t chal[5], const uint8_t rnd[9], bool pre) {
  if (graph_matches(P, pl, pre)) {
    SlotFile sf = make_slotfile(P->n, chal, rnd);
    if (memcmp(&sf, &P->g_sf, sizeof sf)) {
      if (graph_set_arg(P, P->g_first, P->g_first_n, P->g_first_arg, &sf)) {
        drop_graph(P);   // (the runtime would not take the parameter: direct launches)
        return rounds(P, pl, chal, rnd, pre);
      }
      P->g_sf = sf;
    }
    __atomic_store_n((uint32_t*)(P->h_res + 60), 0u, __ATOMIC_SEQ_CST);
    P->seq = P->g_seq;
    PLK_HIP(hipGraphLaunch(P->gx, P->st));
    return PLK_OK;
  }
  drop_graph(P);
  const uint32_t epoch = P->scan_epoch, seq = P->seq;
  // capture ran nothing: anything that keeps this call from a graph runs it with direct launches
  auto direct = [&]() {
    (void)hipGetLastError();
    drop_graph(P);
    P->seq = seq;
    P->scan_epoch = epoch;
    return rounds(P, pl, chal, rnd, pre);
  };
  if (hipStreamBeginCapture(P->st, hipStreamCaptureModeThreadLocal) != hipSuccess) return direct();
  int rc = rounds(P, pl, chal, rnd, pre);
  hipGraph_t g = nullptr;
  const hipError_t e = hipStreamEndCapture(P->st, &g);
  if (rc) {   // (an argument / range error: the same one a direct call reports)
    if (g) (void)hipGraphDestroy(g);
    (void)hipGetLastError();
    P->seq = seq;
    P->scan_epoch = epoch;
    return rc;
  }
  if (e != hipSuccess || !g) {
    if (g) (void)hipGraphDestroy(g);
    return direct();
  }
  P->g = g;
  // per-call state inside the launches (the fused division's scan epochs): no replay
  if (P->scan_epoch != epoch || P->seq != seq + 1) return direct();
  // the first and last kernel nodes, by function
  size_t nn = 0;
  if (hipGraphGetNodes(g, nullptr, &nn) != hipSuccess) return direct();
  std::vector<hipGraphNode_t> nodes(nn);
  if (hipGraphGetNodes(g, nodes.data(), &nn) != hipSuccess) return direct();
  for (hipGraphNode_t nd : nodes) {
    hipGraphNodeType t;
    if (hipGraphNodeGetType(nd, &t) != hipSuccess || t != hipGraphNodeTypeKernel) continue;
    hipKernelNodeParams kp{};
    if (hipGraphKernelNodeGetParams(nd, &kp) != hipSuccess) continue;
    if (kp.func == (void*)prep_kernel) { P->g_first = nd; P->g_first_arg = 1; P->g_first_n = 5; }
    if (kp.func == (void*)scalars_init_kernel) { P->g_first = nd; P->g_first_arg = 0; P->g_first_n = 5; }
    if (kp.func == (void*)commit_pack_kernel || kp.func == (void*)trim_pack_kernel) P->g_last = nd;
  }
  if (!P->g_first || !P->g_last || hipGraphInstantiateWithFlags(&P->gx, g, 0) != hipSuccess) {
    P->gx = nullptr;
    return direct();
  }
  for (int i = 0; i < 13; i++) P->g_pl[i] = pl[i];
  P->g_pre = pre;
  P->g_fix_gen = P->fix_gen;
  for (int o = 1; o < PLK_OPT_COUNT; o++) P->g_opt[o] = plk_opt(o);
  P->g_seq = P->seq;
  P->g_sf = make_slotfile(P->n, chal, rnd);
  PLK_HIP(hipGraphLaunch(P->gx, P->st));   // (this call's launches)
  return PLK_OK;
}

}  // namespace

extern "C" {

int plk_prover_rounds_dev(plk_prover_t* P, const uint8_t* const d_polys[13], const uint8_t chal[5],
                          const uint8_t rand9[9], int flags, uint8_t proof[34]) {
  if (!P || !d_polys || !chal || !rand9) { plk_set_error("plk_prover_rounds_dev: NULL argument"); return PLK_ERR_ARG; }
  for (int i = 0; i < 13; i++)
    if (!d_polys[i]) { plk_set_error("plk_prover_rounds_dev: polynomial %d is NULL", i); return PLK_ERR_ARG; }
  const bool pre = (flags & PLK_PROVE_PREPROCESSED) != 0;
  PROVER_ON_DEVICE(P);
  int rc = P->nhelp                         ? rounds_split(P, d_polys, nullptr, chal, rand9, pre)
           : plk_opt(PLK_OPT_PROVE_GRAPH) ? rounds_graph(P, d_polys, chal, rand9, pre)
                                          : rounds(P, d_polys, chal, rand9, pre);
  if (rc) { (void)hipStreamSynchronize(P->st); return rc; }
  return finish(P, (flags & PLK_PROVE_STRICT) != 0, 0, proof);
}

int plk_prover_profile_dev(plk_prover_t* P, const uint8_t* const d_polys[13], const uint8_t chal[5],
                           const uint8_t rand9[9], int flags, uint8_t proof[34], double ms[4]) {
  if (!P || !d_polys || !chal || !rand9 || !ms) { plk_set_error("plk_prover_profile_dev: NULL argument"); return PLK_ERR_ARG; }
  for (int i = 0; i < 13; i++)
    if (!d_polys[i]) { plk_set_error("plk_prover_profile_dev: polynomial %d is NULL", i); return PLK_ERR_ARG; }
  if (P->nhelp) { plk_set_error("plk_prover_profile_dev: a prover with helpers attached"); return PLK_ERR_ARG; }
  PROVER_ON_DEVICE(P);
  for (hipEvent_t& e : P->tev)
    if (!e) PLK_HIP(hipEventCreate(&e));
  PLK_HIP(hipEventRecord(P->tev[0], P->st));
  P->tev_on = true;
  int rc = rounds(P, d_polys, chal, rand9, (flags & PLK_PROVE_PREPROCESSED) != 0);
  P->tev_on = false;
  if (!rc) rc = hipEventRecord(P->tev[5], P->st) == hipSuccess ? PLK_OK : PLK_ERR_HIP;
  if (rc) { (void)hipStreamSynchronize(P->st); return rc; }
  if ((rc = finish(P, (flags & PLK_PROVE_STRICT) != 0, 0, proof))) return rc;
  PLK_HIP(hipEventSynchronize(P->tev[5]));
  float t[3];
  PLK_HIP(hipEventElapsedTime(&t[0], P->tev[0], P->tev[5]));
  PLK_HIP(hipEventElapsedTime(&t[1], P->tev[1], P->tev[2]));
  PLK_HIP(hipEventElapsedTime(&t[2], P->tev[3], P->tev[4]));
  ms[0] = t[0];
  ms[1] = (double)t[1] + t[2];
  ms[2] = t[1];
  ms[3] = t[2];
  return PLK_OK;
}

int plk_prover_launches(plk_prover_t* P, const uint8_t* const d_polys[13], const uint8_t chal[5], const uint8_t rand9[9],
                        int flags, int* kernels, int* other_nodes) {
  if (!P || !d_polys || !chal || !rand9 || !kernels) { plk_set_error("plk_prover_launches: NULL argument"); return PLK_ERR_ARG; }
  for (int i = 0; i < 13; i++)
    if (!d_polys[i]) { plk_set_error("plk_prover_launches: polynomial %d is NULL", i); return PLK_ERR_ARG; }
  if (P->nhelp) { plk_set_error("plk_prover_launches: a prover with helpers attached"); return PLK_ERR_ARG; }
  PROVER_ON_DEVICE(P);
  PLK_HIP(hipStreamSynchronize(P->st));
  const uint32_t epoch = P->scan_epoch, seq = P->seq;
  PLK_HIP(hipStreamBeginCapture(P->st, hipStreamCaptureModeThreadLocal));
  int rc = rounds(P, d_polys, chal, rand9, (flags & PLK_PROVE_PREPROCESSED) != 0);
  hipGraph_t g = nullptr;
  const hipError_t e = hipStreamEndCapture(P->st, &g);
  P->seq = seq;   // (nothing ran: the next call's completion word and scan epochs are unchanged)
  P->scan_epoch = epoch;
  if (!rc && (e != hipSuccess || !g)) {
    plk_set_error("plk_prover_launches: stream capture failed (%s)", hipGetErrorString(e));
    rc = PLK_ERR_HIP;
  }
  int nk = 0, no = 0;
  size_t nn = 0;
  if (!rc && hipGraphGetNodes(g, nullptr, &nn) == hipSuccess) {
    std::vector<hipGraphNode_t> nodes(nn);
    if (hipGraphGetNodes(g, nodes.data(), &nn) == hipSuccess)
      for (hipGraphNode_t nd : nodes) {
        hipGraphNodeType t;
        if (hipGraphNodeGetType(nd, &t) != hipSuccess) continue;
        if (t == hipGraphNodeTypeKernel) nk++;
        else if (t != hipGraphNodeTypeEmpty) no++;
      }
  }
  if (g) (void)hipGraphDestroy(g);
  (void)hipGetLastError();
  if (rc) return rc;
  *kernels = nk;
  if (other_nodes) *other_nodes = no;
  return PLK_OK;
}

uint64_t plk_prover_alg_bytes(const plk_prover_t* P) { return P ? alg_bytes_for(lens_for(P->n, P->zh_len)) : 0; }

int plk_prover_attach_helpers(plk_prover_t* P, int k) {
  if (!P || k < 0 || k > 2) { plk_set_error("plk_prover_attach_helpers: prover and 0 <= k <= 2 required"); return PLK_ERR_ARG; }
  if (P->dev != plk_cur_device()) {
    plk_set_error("plk_prover_attach_helpers: call from the prover's device %d", P->dev);
    return PLK_ERR_ARG;
  }
  detach_helpers(P);
  if (!k) return PLK_OK;
  int ids[PLK_MAX_SHARDS];
  const int nd = plk_devices(ids, PLK_MAX_SHARDS);
  if (nd < 1 + k) {
    plk_set_error("plk_prover_attach_helpers: %d helper(s) need %d entries in the plk_init_devices list (it has %d)", k,
                  1 + k, nd);
    return PLK_ERR_ARG;
  }
  const Lens L = lens_for(P->n, P->zh_len);
  // helpers need Z_H only (no SRS: they commit nothing): one identity point stands in
  std::vector<uint8_t> zh(P->zh_len);
  PLK_HIP(hipMemcpy(zh.data(), P->d_zh, P->zh_len, hipMemcpyDeviceToHost));
  const uint8_t srs1[3] = {0, 0, 1};
  plk_plonk_desc_t d{};
  d.n = P->n;
  d.z_h = zh.data();
  d.z_h_len = zh.size();
  d.srs_g1 = srs1;
  d.srs_len = 1;
  // chain_assignment (plonkhip/dist.py): one helper takes t_3 (the proving GPU keeps t_2 with its
  // (a b) q_m sum group); two take t_2 and t_3
  const int masks[2][2] = {{PLK_CHAIN_T3, 0}, {PLK_CHAIN_T2, PLK_CHAIN_T3}};
  int rc = PLK_OK;
  for (int h = 0; h < k && !rc; h++) {
    plk_prover* H = nullptr;
    if ((rc = create_on(&d, ids[1 + h], &H))) break;
    P->help[P->nhelp] = H;
    P->help_mask[P->nhelp++] = masks[k - 1][h];
    DevGuard dg;
    if (H->dev != P->dev) {
      int can = 0;   // direct xGMI access both ways where the devices allow it (else staged copies)
      if (hipDeviceCanAccessPeer(&can, H->dev, P->dev) == hipSuccess && can && hipSetDevice(H->dev) == hipSuccess)
        (void)hipDeviceEnablePeerAccess(P->dev, 0);
      if (hipDeviceCanAccessPeer(&can, P->dev, H->dev) == hipSuccess && can && hipSetDevice(P->dev) == hipSuccess)
        (void)hipDeviceEnablePeerAccess(H->dev, 0);
      (void)hipGetLastError();   // (already enabled is not an error here)
    }
    // the helper's input rows: 7 copies of what its chains read + 1 poison row (rounds_split);
    // every byte starts as poison, so an input that is not copied is read as poison, not as stale
    // bytes of an earlier proof (on the same device too: PLK_OPT_PROVE_HELPER_COPY)
    const size_t hb = 8 * hin_stride(P->n);
    if (hipSetDevice(H->dev) != hipSuccess || hipMalloc((void**)&H->hin, hb) != hipSuccess) {
      H->hin = nullptr;
      plk_set_error("plk_prover_attach_helpers: input buffers on device %d", H->dev);
      rc = PLK_ERR_NOMEM;
    } else if (hipMemset(H->hin, 0x05, hb) != hipSuccess) {
      plk_set_error("plk_prover_attach_helpers: input buffers on device %d", H->dev);
      rc = PLK_ERR_HIP;
    }
  }
  if (!rc) {
    const size_t b2 = (L.l2 + 64 + 255) & ~(size_t)255, b3 = (L.l3 + 64 + 255) & ~(size_t)255;
    if (hipMalloc((void**)&P->rx_mem, b2 + b3) != hipSuccess) {
      P->rx_mem = nullptr;
      plk_set_error("plk_prover_attach_helpers: receive buffers");
      rc = PLK_ERR_NOMEM;
    } else {
      P->rx[0] = P->rx_mem;
      P->rx[1] = P->rx_mem + b2;
    }
  }
  if (rc) {
    const std::string why = plk_last_error();
    detach_helpers(P);
    plk_set_error("%s", why.c_str());
  }
  return rc;
}

int plk_prover_helpers(const plk_prover_t* P) { return P ? P->nhelp : 0; }

int plk_prover_rounds_multi_dev(plk_prover_t* P, const uint8_t* const* d_polys, int ndev, const uint8_t chal[5],
                                const uint8_t rand9[9], int flags, uint8_t proof[34]) {
  if (!P || !d_polys || !chal || !rand9) { plk_set_error("plk_prover_rounds_multi_dev: NULL argument"); return PLK_ERR_ARG; }
  if (ndev != 1 + P->nhelp) {
    plk_set_error("plk_prover_rounds_multi_dev: %d input sets for 1 + %d devices", ndev, P->nhelp);
    return PLK_ERR_ARG;
  }
  for (int i = 0; i < 13 * ndev; i++)
    if (!d_polys[i]) { plk_set_error("plk_prover_rounds_multi_dev: polynomial %d of set %d is NULL", i % 13, i / 13); return PLK_ERR_ARG; }
  const bool pre = (flags & PLK_PROVE_PREPROCESSED) != 0;
  PROVER_ON_DEVICE(P);
  int rc = P->nhelp ? rounds_split(P, d_polys, d_polys, chal, rand9, pre) : rounds(P, d_polys, chal, rand9, pre);
  if (rc) { (void)hipStreamSynchronize(P->st); return rc; }
  return finish(P, (flags & PLK_PROVE_STRICT) != 0, 0, proof);
}

size_t plk_prover_chain_bytes(const plk_prover_t* P, int which) {
  if (!P || (which != PLK_CHAIN_T2 && which != PLK_CHAIN_T3)) return 0;
  const Lens L = lens_for(P->n, P->zh_len);
  return (size_t)(which == PLK_CHAIN_T2 ? L.l2 : L.l3) + 64;   // (the numerator reads whole dwords)
}

namespace {
int check_chain_args(const char* fn, const plk_prover_t* P, const uint8_t* const* d_polys, const uint8_t* chal,
                     const uint8_t* rand9, int which, const void* t2, const void* t3) {
  if (!P || !d_polys || !chal || !rand9) { plk_set_error("%s: NULL argument", fn); return PLK_ERR_ARG; }
  for (int i = 0; i < 13; i++)
    if (!d_polys[i]) { plk_set_error("%s: polynomial %d is NULL", fn, i); return PLK_ERR_ARG; }
  if (which & ~(PLK_CHAIN_T2 | PLK_CHAIN_T3)) { plk_set_error("%s: bad chain mask %d", fn, which); return PLK_ERR_ARG; }
  if (((which & PLK_CHAIN_T2) && !t2) || ((which & PLK_CHAIN_T3) && !t3)) {
    plk_set_error("%s: NULL chain buffer", fn);
    return PLK_ERR_ARG;
  }
  if (((uintptr_t)t2 | (uintptr_t)t3) % 16) { plk_set_error("%s: chain buffers must be 16-byte aligned", fn); return PLK_ERR_ARG; }
  return PLK_OK;
}
// records an event on `from` and makes `to` wait for it (cross-stream, same device)
int stream_after(hipStream_t to, hipStream_t from, hipEvent_t ev) {
  PLK_HIP(hipEventRecord(ev, from));
  PLK_HIP(hipStreamWaitEvent(to, ev, 0));
  return PLK_OK;
}
}  // namespace

int plk_prover_chains_dev(plk_prover_t* P, const uint8_t* const d_polys[13], const uint8_t chal[5],
                          const uint8_t rand9[9], int which, uint8_t* d_t2, uint8_t* d_t3, void* done) {
  int rc = check_chain_args("plk_prover_chains_dev", P, d_polys, chal, rand9, which, d_t2, d_t3);
  if (rc) return rc;
  if (!which) return PLK_OK;
  PROVER_ON_DEVICE(P);
  // write-after-read: the previous call's d_t2 / d_t3 may still be read by work on `done` (e.g.
  // an RCCL send of the last products): this call's products are written only after it
  if ((rc = stream_after(P->st, (hipStream_t)done, P->ev))) return rc;
#if PLK_DIAG_DROP_HANDOFF & 1
  // diagnostic build: the products are poisoned first and written ~20 ms later, so a consumer
  // with no ordering behind this call reads poison however the streams are scheduled in time
  if (d_t2) PLK_HIP(hipMemsetAsync(d_t2, 0x05, plk_prover_chain_bytes(P, PLK_CHAIN_T2), P->st));
  if (d_t3) PLK_HIP(hipMemsetAsync(d_t3, 0x05, plk_prover_chain_bytes(P, PLK_CHAIN_T3), P->st));
  hipLaunchKernelGGL(diag_spin_kernel, dim3(1), dim3(64), 0, P->st, 2000000ull);
  PLK_HIP(hipGetLastError());
#endif
  RoundsMode md;
  md.only = which;
  md.o2 = d_t2;
  md.o3 = d_t3;
  rc = rounds(P, d_polys, chal, rand9, false, md);
  if (rc) { (void)hipStreamSynchronize(P->st); return rc; }
#if PLK_DIAG_DROP_HANDOFF & 1   // diagnostic build only (tests/test_split_streams_gpu.py): no ordering
  return PLK_OK;
#endif
  return stream_after((hipStream_t)done, P->st, P->ev);   // (NULL: the null stream, torch's default)
}

int plk_prover_rounds_ext_dev(plk_prover_t* P, const uint8_t* const d_polys[13], const uint8_t chal[5],
                              const uint8_t rand9[9], int flags, int which, const uint8_t* d_t2, const uint8_t* d_t3,
                              void* ready, uint8_t proof[34]) {
  int rc = check_chain_args("plk_prover_rounds_ext_dev", P, d_polys, chal, rand9, which, d_t2, d_t3);
  if (rc) return rc;
  PROVER_ON_DEVICE(P);
  RoundsMode md;
  md.ext = which;
  md.t2 = d_t2;
  md.t3 = d_t3;
  if (which && !(PLK_DIAG_DROP_HANDOFF & 2)) {   // everything enqueued on `ready` so far (the bytes'
    PLK_HIP(hipEventRecord(P->ev, (hipStream_t)ready));   // arrival; NULL: the null stream) before they are read
    md.ready[0] = P->ev;
  }
  rc = rounds(P, d_polys, chal, rand9, (flags & PLK_PROVE_PREPROCESSED) != 0, md);
  if (rc) { (void)hipStreamSynchronize(P->st); return rc; }
  return finish(P, (flags & PLK_PROVE_STRICT) != 0, 0, proof);
}

int plk_prover_preprocess(plk_prover_t* P, const uint8_t* const d_polys[13]) {
  if (!P) { plk_set_error("plk_prover_preprocess: NULL prover"); return PLK_ERR_ARG; }
  PROVER_ON_DEVICE(P);
  PLK_HIP(hipStreamSynchronize(P->st));   // (no round may still read the old transforms)
  ++P->fix_gen;                            // (a captured proof graph reads the old ones: recapture)
  for (auto& f : P->fix) f = plk_prover::Fixed{};
  (void)hipFree(P->fix_mem);
  P->fix_mem = nullptr;
  if (!d_polys) return PLK_OK;   // dropped
  const uint64_t n = P->n;
  const Lens L = lens_for(n, P->zh_len);
  // the round-3 products with a fixed b (rounds(): g1[0..3], g1[5], g2[0]) and their a
  // operands' upper-bound lengths
  const int which[] = {5, 6, 3, 12, 10, 4};   // q_l q_r q_o l_1_x s_sigma_3 q_m
  const uint64_t la[] = {L.la, L.la, L.la, L.lz1, L.lzx, L.lab};
  size_t words = 0;
  int ks[6], fs[6];
  for (int i = 0; i < 6; i++) {
    if (!d_polys[which[i]]) { plk_set_error("plk_prover_preprocess: polynomial %d is NULL", which[i]); return PLK_ERR_ARG; }
    ks[i] = plk_poly_mul_transform_plan(la[i], n, &fs[i]);
    if (ks[i] > 0) words += (size_t)1 << ks[i];
  }
  if (!words) return PLK_OK;   // (small circuits: no product runs through the transform engine)
  if (hipMalloc((void**)&P->fix_mem, 4 * words) != hipSuccess) {
    P->fix_mem = nullptr;
    plk_set_error("plk_prover_preprocess: hipMalloc(%zu) failed", 4 * words);
    return PLK_ERR_NOMEM;
  }
  uint32_t* t = P->fix_mem;
  for (int i = 0; i < 6; i++) {
    if (ks[i] <= 0) continue;
    const int rc = plk_poly_mul_pretransform(d_polys[which[i]], n, ks[i], fs[i], t, P->st);
    if (rc) {
      plk_prover_preprocess(P, nullptr);
      return rc;
    }
    P->fix[which[i]] = plk_prover::Fixed{d_polys[which[i]], t, ks[i], fs[i]};
    t += (size_t)1 << ks[i];
  }
  PLK_HIP(hipStreamSynchronize(P->st));
  return PLK_OK;
}

int plk_prover_prove(plk_prover_t* P, const plk_circuit_t* c, const uint8_t chal[5], const uint8_t rand9[9],
                     uint8_t proof[34]) {
  if (!P || !c || !chal || !rand9) { plk_set_error("plk_prover_prove: NULL argument"); return PLK_ERR_ARG; }
  if (!P->have_circuit_tables) {
    plk_set_error("plk_prover_prove: prover created without h / k1_h / k2_h / h_pows_inv");
    return PLK_ERR_ARG;
  }
  PROVER_ON_DEVICE(P);
  const uint64_t n = P->n;
  const uint8_t* parts[11] = {c->q_m, c->q_l, c->q_r, c->q_o, c->q_c, c->copy_a, c->copy_b, c->copy_c, c->a, c->b, c->c};
  for (int i = 0; i < 11; i++)
    if (!parts[i]) { plk_set_error("plk_prover_prove: circuit array %d is NULL", i); return PLK_ERR_ARG; }
  // upload: q_m q_l q_r q_o q_c | copy_a copy_b copy_c (2n each) | a b c
  std::vector<uint8_t> h(14 * n);
  memcpy(&h[0], c->q_m, n); memcpy(&h[n], c->q_l, n); memcpy(&h[2 * n], c->q_r, n); memcpy(&h[3 * n], c->q_o, n);
  memcpy(&h[4 * n], c->q_c, n);
  memcpy(&h[5 * n], c->copy_a, 2 * n); memcpy(&h[7 * n], c->copy_b, 2 * n); memcpy(&h[9 * n], c->copy_c, 2 * n);
  memcpy(&h[11 * n], c->a, n); memcpy(&h[12 * n], c->b, n); memcpy(&h[13 * n], c->c, n);
  for (size_t i = 0; i < 14 * n; i++)
    if (!(i >= 5 * n && i < 11 * n)) h[i] %= HFP;   // HF values (hf_new reduces), copies stay raw
  PLK_HIP(hipMemcpyAsync(P->d_cir, h.data(), h.size(), hipMemcpyHostToDevice, P->st));
  // challenges are needed by the grand product before rounds() uploads the scalar file
  SlotFile sf0{};
  uint8_t* S0 = sf0.b;
  S0[S_ONE] = 1; S0[S_NEG1] = 16;
  S0[S_ALPHA] = chal[0] % HFP; S0[S_BETA] = chal[1] % HFP; S0[S_GAMMA] = chal[2] % HFP;
  S0[S_Z] = chal[3] % HFP; S0[S_V] = chal[4] % HFP;
  S0[S_OMEGA] = 4; S0[S_K1] = 2; S0[S_K2] = 3;
  S0[S_ACCW + 1] = h_pow(4, n);   // x = omega^n for the acc_x(omega^n) == 1 check below
  hipLaunchKernelGGL(scalars_init_kernel, dim3(1), dim3(NSLOT), 0, P->st, sf0, P->d_S, P->d_stat, (int)ST_GATE,
                     (int)NSTAT);
  PLK_HIP(hipGetLastError());
  // stage A: checks + sigma, 11 interpolations, grand product, acc_x and L1(x)
  for (int i = 0; i < 13; i++) PLK_HIP(hipMemsetAsync(P->d_polys[i], 0, n, P->st));
  hipLaunchKernelGGL(circuit_check_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, P->st, P->d_cir, n,
                     P->d_h3, P->d_vals, P->d_stat);
  PLK_HIP(hipGetLastError());
  hipLaunchKernelGGL(interpolate_kernel, dim3((unsigned)((11 * n + 255) / 256)), dim3(256), 0, P->st, P->d_hinv, n,
                     P->d_vals, 11, P->d_outs);
  PLK_HIP(hipGetLastError());
  hipLaunchKernelGGL(grand_product_kernel, dim3(1), dim3(64), 0, P->st, P->d_vals, n,
                     (const uint8_t* const*)P->d_outs, P->d_S, P->ACCV);
  PLK_HIP(hipGetLastError());
  hipLaunchKernelGGL(unit_vector_kernel, dim3(1), dim3(256), 0, P->st, P->E0, n);
  PLK_HIP(hipGetLastError());
  // acc_x and L1(x) = interpolate_at_h(e_0) (src/plonk.h:362, 381-387)
  hipLaunchKernelGGL(interpolate_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, P->st, P->d_hinv, n,
                     P->ACCV, 1, P->d_outs + 11);
  PLK_HIP(hipGetLastError());
  hipLaunchKernelGGL(interpolate_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, P->st, P->d_hinv, n,
                     P->E0, 1, P->d_outs + 12);
  PLK_HIP(hipGetLastError());
  // acc_x(omega^n) must be 1 (src/plonk.h:366-368): evaluated straight into its status word
  {
    const int erc = evals(P, {{P->d_polys[11], n, S_ACCW + 1, S_ACCW}}, EV_POST_ACC);
    if (erc) { (void)hipStreamSynchronize(P->st); return erc; }
  }

  const uint8_t* pl[13];
  for (int i = 0; i < 13; i++) pl[i] = P->d_polys[i];
  int rc = P->nhelp ? rounds_split(P, pl, nullptr, chal, rand9, false) : rounds(P, pl, chal, rand9);
  if (rc) { (void)hipStreamSynchronize(P->st); return rc; }
  return finish(P, 1, 1, proof);
}

}  // extern "C"
