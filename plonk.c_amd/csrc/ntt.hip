// Exact GF(17) polynomial multiplication (reference poly_mul, src/poly.h:106-122) on gfx950.
//
// GF(17)* has order 16, so GF(17) itself has no NTT beyond 16 points.  The product of two
// coefficient vectors reduced into [0,17) is an integer convolution whose terms are all
// < min(la, lb) * 256, which is < p = 2013265921 (BabyBear, 2-adicity 27) whenever
// min(la, lb) < 7,864,320.  So the convolution is computed EXACTLY by an NTT over BabyBear
// (Montgomery u32) and reduced mod 17 at the end: bit-identical to the schoolbook.
//
// Transform layout -- no bit-reversal pass anywhere:
//   forward  DIF (Gentleman-Sande), natural order in  -> bit-reversed out
//   pointwise product in bit-reversed order
//   inverse  DIT (Cooley-Tukey),   bit-reversed in   -> natural order out, times N^-1
// A size-2^k transform is cut into passes over disjoint bit ranges [lo, lo+M) of the index;
// one pass = one launch whose workgroups each own a tile of 2^M rows (the butterfly bits)
// x C columns (consecutive low-bit values when lo > 0, consecutive groups when lo = 0),
// staged once through LDS and run through all M radix-2 stages there.
// Twiddles factor into a universal per-stage table T[2^j + r] = w_{2^(j+1)}^r (independent
// of N) times a per-column factor F[c][j] = w_{2^27}^(L * 2^(26-lo-j)) (1 when lo = 0).
//
// poly_mul plan at 2^k > 2^12 (3 launches for k <= 23):
//   ntt_pass_kernel   forward passes over the high bits, reading the u8 inputs directly
//   ntt_center_kernel last forward pass (lo = 0) of a AND b, pointwise product, first
//                     inverse pass -- one tile, one LDS round trip
//   ntt_pass_kernel   inverse passes over the high bits; the last one scales by N^-1,
//                     leaves Montgomery form, reduces mod 17, stores bytes and records the
//                     last non-zero index for the reference's trailing-zero trim
// k <= 12: one workgroup does everything (polymul_small_kernel); min(la, lb) <= 32: direct
// convolution (polymul_direct_kernel).
#include "plk_device.h"
#include "plk_internal.h"

#include <chrono>

#include <stdio.h>
#include <stdlib.h>

#include <algorithm>
#include <vector>

__constant__ uint32_t c_mont17[17];            // v * R mod p for v = 0..16

namespace {

constexpr int NTT_THREADS = 512;
constexpr int PAD = 4;

// LDS row padding: one spare word after every 32 rows, so the strided element accesses of
// the low-stride rounds (lanes at base = 2^R g) hit distinct banks instead of 2^R-way
// conflicts.  Column stride RS = phys(rows) + PAD.
__device__ __forceinline__ int phys(int r) { return r + (r >> 5); }
__host__ __device__ constexpr int col_stride(int rows) { return rows + (rows >> 5) + PAD; }

struct Tw {
  const uint32_t* small;   // T[2^j + r] = w_{2^(j+1)}^r  (Montgomery), 2^PLK_NTT_SMALL_LOG
  const uint32_t* lo;      // w_{2^27}^i,        i < 4096
  const uint32_t* hi;      // w_{2^27}^(4096 i), i < 2^15
};

__device__ __forceinline__ uint32_t root27(const Tw& t, uint32_t e) {  // w_{2^27}^e, e < 2^27
  return bb::mmul(t.lo[e & 4095u], t.hi[e >> 12]);
}

// Tile geometry of one pass
struct Pass {
  int k;       // log2 N
  int lo;      // lowest bit of this pass
  int M;       // bits in this pass (rows = 2^M)
  int C;       // columns per tile (power of two; >= 4 when lo > 0)
};

// global index of (row r, column c) of tile t
__device__ __forceinline__ uint64_t tile_index(const Pass& p, uint32_t t, int r, int c) {
  if (p.lo == 0) return (((uint64_t)t * p.C + c) << p.M) | (uint64_t)r;
  const uint32_t per_h = (1u << p.lo) / p.C;
  const uint64_t H = t / per_h;
  const uint32_t L = (t % per_h) * p.C + c;
  return (H << (p.lo + p.M)) | ((uint64_t)r << p.lo) | L;
}

// F[c][j] = w_{2^27}^(L * 2^(26-lo-j)) for the tile's columns (only when lo > 0)
__device__ void column_factors(const Pass& p, uint32_t t, const Tw& tw, uint32_t* F) {
  if (p.lo == 0) return;
  const uint32_t per_h = (1u << p.lo) / p.C;
  for (int c = threadIdx.x; c < p.C; c += blockDim.x) {
    const uint32_t L = (t % per_h) * p.C + c;
    uint32_t f = root27(tw, L << (27 - p.lo - p.M));      // stage j = M-1
    for (int j = p.M - 1; j >= 0; j--) {
      F[c * p.M + j] = f;
      f = bb::mmul(f, f);
    }
  }
}

// ---- global <-> LDS tile movement, 4 elements per thread-step --------------------------
// lo == 0: the tile is C contiguous runs of 2^M; 4 consecutive rows of one column.
// lo  > 0: rows of C contiguous elements; 4 consecutive columns of one row.
// LDS layout X[c * RS + phys(r)], RS = col_stride(2^M).
template <bool U8>
__device__ __forceinline__ void load_tile(const Pass& p, uint32_t t, uint32_t* X, int RS, const uint32_t* d,
                                          const uint8_t* s8, uint64_t ls) {
  const int rows = 1 << p.M;
  if (p.lo == 0 && p.M < 2) {                  // tiny single-pass transforms
    for (int e = threadIdx.x; e < rows * p.C; e += blockDim.x) {
      const int r = e & (rows - 1), c = e >> p.M;
      const uint64_t idx = tile_index(p, t, r, c);
      X[c * RS + phys(r)] = U8 ? (idx < ls ? c_mont17[s8[idx] % 17u] : 0u) : d[idx];
    }
    return;
  }
  const int E4 = (rows * p.C) >> 2;
  for (int e = threadIdx.x; e < E4; e += blockDim.x) {
    int r, c;
    bool colrun;
    if (p.lo == 0) { c = (4 * e) >> p.M; r = (4 * e) & (rows - 1); colrun = true; }
    else { r = (4 * e) / p.C; c = (4 * e) % p.C; colrun = false; }
    const uint64_t idx = tile_index(p, t, r, c);
    uint32_t v[4];
    if (U8) {
#pragma unroll
      for (int i = 0; i < 4; i++) v[i] = idx + i < ls ? c_mont17[s8[idx + i] % 17u] : 0u;
    } else {
      const uint4 q = *reinterpret_cast<const uint4*>(d + idx);
      v[0] = q.x; v[1] = q.y; v[2] = q.z; v[3] = q.w;
    }
    if (colrun) {
#pragma unroll
      for (int i = 0; i < 4; i++) X[c * RS + phys(r) + i] = v[i];   // r % 4 == 0: one 32-row block
    } else {
#pragma unroll
      for (int i = 0; i < 4; i++) X[(c + i) * RS + phys(r)] = v[i];
    }
  }
}

__device__ __forceinline__ void store_tile(const Pass& p, uint32_t t, const uint32_t* X, int RS, uint32_t* d) {
  const int rows = 1 << p.M;
  if (p.lo == 0 && p.M < 2) {
    for (int e = threadIdx.x; e < rows * p.C; e += blockDim.x) {
      const int r = e & (rows - 1), c = e >> p.M;
      d[tile_index(p, t, r, c)] = X[c * RS + phys(r)];
    }
    return;
  }
  const int E4 = (rows * p.C) >> 2;
  for (int e = threadIdx.x; e < E4; e += blockDim.x) {
    int r, c;
    uint4 q;
    if (p.lo == 0) {
      c = (4 * e) >> p.M; r = (4 * e) & (rows - 1);
      const uint32_t* x = X + c * RS + phys(r);
      q = make_uint4(x[0], x[1], x[2], x[3]);
    } else {
      r = (4 * e) / p.C; c = (4 * e) % p.C;
      const int pr = phys(r);
      q = make_uint4(X[c * RS + pr], X[(c + 1) * RS + pr], X[(c + 2) * RS + pr], X[(c + 3) * RS + pr]);
    }
    *reinterpret_cast<uint4*>(d + tile_index(p, t, r, c)) = q;
  }
}

// ---- radix-2^R rounds in registers -------------------------------------------------------
// DIF stages j, j-1, .., j-R+1 on the 2^R elements {base + k 2^(j-R+1)} of one column:
// (u, v) -> (u + v, (u - v) w), w = T[2^s + (row mod 2^s)] (* F[c][s] when lo > 0).
template <int R, bool INV>
__device__ __forceinline__ void round_r(uint32_t* X, int M, int C, int RS, int top, const uint32_t* Tsm,
                                       const uint32_t* F, bool has_f) {
  constexpr int NE = 1 << R;
  const int lowbit = INV ? top : top - R + 1;      // lowest stage bit of this round
  const int hstride = 1 << lowbit;
  const int ng = C << (M - R);
  for (int gi = threadIdx.x; gi < ng; gi += blockDim.x) {
    const int c = gi >> (M - R);
    const int g = gi & ((1 << (M - R)) - 1);
    const int base = (g & (hstride - 1)) | ((g >> lowbit) << (lowbit + R));
    uint32_t* col = X + c * RS;
    uint32_t v[NE];
#pragma unroll
    for (int k = 0; k < NE; k++) v[k] = col[phys(base + k * hstride)];
#pragma unroll
    for (int t = 0; t < R; t++) {
      const int kb = INV ? t : (R - 1 - t);          // k-bit of this stage
      const int s = lowbit + kb;                     // stage = row bit
      const int hk = 1 << kb;
#pragma unroll
      for (int k = 0; k < NE; k++) {
        if (k & hk) continue;
        const int rr = (base + k * hstride) & ((1 << s) - 1);
        uint32_t w = Tsm[(1 << s) + rr];
        if (has_f) w = bb::mmul(w, F[c * M + s]);
        const uint32_t u = v[k], x = v[k + hk];
        if (!INV) {
          v[k] = bb::madd(u, x);
          v[k + hk] = bb::mmul(bb::msub(u, x), w);
        } else {
          const uint32_t xw = bb::mmul(x, w);
          v[k] = bb::madd(u, xw);
          v[k + hk] = bb::msub(u, xw);
        }
      }
    }
#pragma unroll
    for (int k = 0; k < NE; k++) col[phys(base + k * hstride)] = v[k];
  }
  __syncthreads();
}

// All M stages of a tile: DIF top-down / DIT bottom-up, in rounds of up to 4 stages.
template <bool INV>
__device__ void tile_stages(uint32_t* X, int M, int C, int RS, const uint32_t* Tsm, const uint32_t* F,
                            bool has_f) {
  int done = 0;
  while (done < M) {
    const int left = M - done;
    const int R = left >= 4 ? 4 : left;
    const int top = INV ? done : (M - 1 - done);
    switch (R) {
      case 4: round_r<4, INV>(X, M, C, RS, top, Tsm, F, has_f); break;
      case 3: round_r<3, INV>(X, M, C, RS, top, Tsm, F, has_f); break;
      case 2: round_r<2, INV>(X, M, C, RS, top, Tsm, F, has_f); break;
      default: round_r<1, INV>(X, M, C, RS, top, Tsm, F, has_f); break;
    }
    done += R;
  }
}

}  // namespace


// Input/output modes of a pass
enum : int { IN_U32 = 0, IN_U8 = 1 };
enum : int { OUT_U32 = 0, OUT_U8 = 1 };

// One NTT pass over 1 or 2 arrays (blockIdx.y).  IN_U8: arrays are byte vectors of length
// la / lb (zero-padded, reduced mod 17, converted to Montgomery).  OUT_U8: the final inverse
// pass: scale by N^-1 given in normal form (which also leaves Montgomery form), mod 17,
// bytes to out8 for idx < out_len; max non-zero idx + 1 -> *nz (atomicMax).
template <bool INV, int IN, int OUT>
__global__ __launch_bounds__(NTT_THREADS) void ntt_pass_kernel(
    Pass p, uint32_t* d0, uint32_t* d1, const uint8_t* a8, const uint8_t* b8, uint64_t la, uint64_t lb,
    Tw tw, uint8_t* out8, uint64_t out_len, uint32_t ninv, uint32_t* nz) {
  extern __shared__ __attribute__((aligned(16))) uint32_t smem[];
  const int rows = 1 << p.M;
  const int RS = col_stride(rows);
  uint32_t* X = smem;
  uint32_t* Tsm = X + p.C * RS;
  uint32_t* F = Tsm + rows;
  uint32_t* d = blockIdx.y == 0 ? d0 : d1;
  const uint32_t t = blockIdx.x;

  for (int i = threadIdx.x; i < rows; i += blockDim.x) Tsm[i] = tw.small[i];
  column_factors(p, t, tw, F);
  if (IN == IN_U8) load_tile<true>(p, t, X, RS, nullptr, blockIdx.y == 0 ? a8 : b8, blockIdx.y == 0 ? la : lb);
  else load_tile<false>(p, t, X, RS, d, nullptr, 0);
  __syncthreads();
  tile_stages<INV>(X, p.M, p.C, RS, Tsm, F, p.lo != 0);

  if (OUT == OUT_U32) {
    store_tile(p, t, X, RS, d);
    return;
  }
  uint32_t last = 0;
  const int E = rows * p.C;
  for (int e = threadIdx.x; e < E; e += blockDim.x) {
    int r, c;
    if (p.lo == 0) { r = e & (rows - 1); c = e >> p.M; }
    else { c = e % p.C; r = e / p.C; }
    const uint64_t idx = tile_index(p, t, r, c);
    if (idx < out_len) {
      const uint8_t byte = (uint8_t)(bb::mmul(X[c * RS + phys(r)], ninv) % 17u);
      out8[idx] = byte;
      if (byte && (uint32_t)idx + 1 > last) last = (uint32_t)idx + 1;
    }
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) last = max(last, (uint32_t)__shfl_xor(last, off, PLK_WAVE));
  if ((threadIdx.x & (PLK_WAVE - 1)) == 0 && last) atomicMax(nz, last);
}

// Whole poly_mul in one workgroup for N = 2^k <= 2^PLK_SMALL_LOG.
__global__ __launch_bounds__(1024) void polymul_small_kernel(const uint8_t* a8, uint64_t la, const uint8_t* b8,
                                                             uint64_t lb, int k, Tw twf, Tw twi,
                                                             uint8_t* out8, uint32_t ninv, uint32_t* nz) {
  extern __shared__ __attribute__((aligned(16))) uint32_t smem[];
  const int N = 1 << k;
  const int RS = col_stride(N);
  uint32_t* X = smem;
  uint32_t* Y = X + RS;
  uint32_t* Tf = Y + RS;
  uint32_t* Ti = Tf + N;
  for (int i = threadIdx.x; i < N; i += blockDim.x) {
    X[phys(i)] = i < (int64_t)la ? c_mont17[a8[i] % 17] : 0u;
    Y[phys(i)] = i < (int64_t)lb ? c_mont17[b8[i] % 17] : 0u;
    Tf[i] = twf.small[i];
    Ti[i] = twi.small[i];
  }
  __syncthreads();
  if (k > 0) {
    tile_stages<false>(X, k, 1, RS, Tf, nullptr, false);
    tile_stages<false>(Y, k, 1, RS, Tf, nullptr, false);
  }
  for (int i = threadIdx.x; i < N; i += blockDim.x) X[phys(i)] = bb::mmul(X[phys(i)], Y[phys(i)]);
  __syncthreads();
  if (k > 0) tile_stages<true>(X, k, 1, RS, Ti, nullptr, false);
  const uint64_t rl = la + lb - 1;
  uint32_t last = 0;
  for (int i = threadIdx.x; i < N; i += blockDim.x) {
    if ((uint64_t)i < rl) {
      const uint8_t byte = (uint8_t)(bb::mmul(X[phys(i)], ninv) % 17u);
      out8[i] = byte;
      if (byte) last = max(last, (uint32_t)i + 1);
    }
  }
  last = plk_block_max(last);
  if (threadIdx.x == 0 && nz) *nz = last;
}

// Trimmed length of out8[0, rl): index + 1 of the last non-zero byte, 0 if none (the
// reference's poly_new trim, src/poly.h:21-24).  One block scans backwards in 16 KiB chunks and
// stops at the first chunk holding a non-zero byte -- almost always the last one -- instead
// of every tile of the product racing on one atomic word.
__global__ __launch_bounds__(1024) void trim_kernel(const uint8_t* __restrict__ out8, uint64_t rl, uint32_t* nz) {
  constexpr int64_t CH = 16384;
  for (int64_t end = (int64_t)rl; end > 0; end -= CH) {
    const int64_t start = end > CH ? end - CH : 0;
    uint32_t last = 0;
    for (int64_t i = start + threadIdx.x; i < end; i += blockDim.x)
      if (out8[i]) last = max(last, (uint32_t)(i + 1));
    last = plk_block_max(last);
    if (last) {
      if (threadIdx.x == 0) *nz = last;
      return;
    }
  }
  if (threadIdx.x == 0) *nz = 0;
}

int plk_trim_launch(const uint8_t* d, uint64_t len, uint32_t* d_nz, hipStream_t st) {
  hipLaunchKernelGGL(trim_kernel, dim3(1), dim3(1024), 0, st, d, len, d_nz);
  PLK_HIP(hipGetLastError());
  return PLK_OK;
}

// Direct convolution when one operand is short: out[i] = sum_j a[j] b[i-j] mod 17 over the
// short operand s (length ls <= 32, staged in LDS), the long one read coalesced.
__global__ __launch_bounds__(256) void polymul_direct_kernel(const uint8_t* lg, uint64_t llg, const uint8_t* sh,
                                                             int lsh, uint8_t* out8, uint32_t* nz) {
  __shared__ uint32_t S[64];
  if ((int)threadIdx.x < lsh) S[threadIdx.x] = sh[threadIdx.x] % 17u;
  __syncthreads();
  const uint64_t rl = llg + lsh - 1;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < rl; i += (uint64_t)gridDim.x * blockDim.x) {
    uint32_t acc = 0;
    for (int j = 0; j < lsh; j++) {
      const int64_t o = (int64_t)i - j;
      if (o >= 0 && (uint64_t)o < llg) acc += S[j] * (lg[o] % 17u);
    }
    out8[i] = (uint8_t)(acc % 17u);
  }
  (void)nz;   // trimmed length: trim_kernel
}

// ------------------------------------------------------------------------------ host side
// Root tables live on every device that runs transforms (the primary of plk_init, and the helper
// devices of a multi-device prover, plk_prover_attach_helpers): one set per device id, picked by
// the calling thread's current device at launch.
namespace {

struct TwHost {
  uint32_t* d_small_f = nullptr;
  uint32_t* d_small_i = nullptr;
  uint32_t* d_lo_f = nullptr;
  uint32_t* d_hi_f = nullptr;
  uint32_t* d_lo_i = nullptr;
  uint32_t* d_hi_i = nullptr;
};
struct DevTw {
  TwHost bb, f29;
};
DevTw g_tw[PLK_MAX_DEVICES];

DevTw& cur_tw() { return g_tw[plk_cur_device()]; }
Tw tw_fwd() { const TwHost& t = cur_tw().bb; return Tw{t.d_small_f, t.d_lo_f, t.d_hi_f}; }
Tw tw_inv() { const TwHost& t = cur_tw().bb; return Tw{t.d_small_i, t.d_lo_i, t.d_hi_i}; }
PlkTwTables to_tables(const TwHost& t) {
  return PlkTwTables{t.d_small_f, t.d_small_i, t.d_lo_f, t.d_hi_f, t.d_lo_i, t.d_hi_i};
}
void free_tw(TwHost& t) {
  for (uint32_t* p : {t.d_small_f, t.d_small_i, t.d_lo_f, t.d_hi_f, t.d_lo_i, t.d_hi_i}) (void)hipFree(p);
  t = TwHost{};
}

}  // namespace

static int64_t g_marks[16];
void plk_host_mark(int id) {
  if (id >= 0 && id < 16 && (id == 0 || !g_marks[id]))   // (the first time of each point after mark 0)
    g_marks[id] = std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now().time_since_epoch()).count();
}
void plk_host_marks_print(void) {
  fprintf(stderr, "host marks (us from mark 0):");
  for (int i = 1; i < 16; i++)
    if (g_marks[i]) fprintf(stderr, " %d:%.1f", i, (g_marks[i] - g_marks[0]) / 1e3);
  fprintf(stderr, "\n");
  for (int i = 0; i < 16; i++) g_marks[i] = 0;
}

int plk_cur_device(void) {
  int d = 0;
  if (hipGetDevice(&d) != hipSuccess || d < 0 || d >= PLK_MAX_DEVICES) d = 0;
  return d;
}

PlkTwTables plk_ntt_tables29(void) { return to_tables(cur_tw().f29); }
PlkTwTables plk_ntt_tables(void) { return to_tables(cur_tw().bb); }

// the tables of the CURRENT device (idempotent per device)
int plk_ntt_init_tables(void) {
  const int dev = plk_cur_device();
  TwHost& T = g_tw[dev].bb;
  TwHost& T29 = g_tw[dev].f29;
  if (T.d_small_f) return PLK_OK;
  // tiles of 2^12 rows with two arrays exceed the default 64 KB dynamic-LDS limit
  const int lds_max = 150 * 1024;   // leaves room for the kernels' static LDS
  PLK_HIP(hipFuncSetAttribute((const void*)polymul_small_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, lds_max));
  PLK_HIP(hipFuncSetAttribute((const void*)ntt_pass_kernel<false, IN_U32, OUT_U32>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, lds_max));
  PLK_HIP(hipFuncSetAttribute((const void*)ntt_pass_kernel<true, IN_U32, OUT_U32>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, lds_max));
  const uint32_t w27 = bb::hpow(bb::GENERATOR, (bb::P - 1) >> bb::TWO_ADICITY);   // order 2^27
  const uint32_t w27i = bb::hpow(w27, bb::P - 2);
  const int SM = 1 << PLK_NTT_SMALL_LOG;
  std::vector<uint32_t> sf(SM), si(SM), lf(4096), hf(1 << 15), li(4096), hi_(1 << 15);
  sf[0] = si[0] = bb::to_mont(1);
  for (int j = 0; (1 << j) < SM; j++) {
    const uint32_t wf = bb::hpow(w27, 1ull << (26 - j));   // order 2^(j+1)
    const uint32_t wi = bb::hpow(w27i, 1ull << (26 - j));
    uint64_t xf = 1, xi = 1;
    for (int r = 0; r < (1 << j); r++) {
      sf[(1 << j) + r] = bb::to_mont((uint32_t)xf);
      si[(1 << j) + r] = bb::to_mont((uint32_t)xi);
      xf = xf * wf % bb::P;
      xi = xi * wi % bb::P;
    }
  }
  {
    uint64_t x = 1, y = 1;
    for (int i = 0; i < 4096; i++) {
      lf[i] = bb::to_mont((uint32_t)x);
      li[i] = bb::to_mont((uint32_t)y);
      x = x * w27 % bb::P;
      y = y * w27i % bb::P;
    }
    const uint64_t s = bb::hpow(w27, 4096), si2 = bb::hpow(w27i, 4096);
    x = 1, y = 1;
    for (int i = 0; i < (1 << 15); i++) {
      hf[i] = bb::to_mont((uint32_t)x);
      hi_[i] = bb::to_mont((uint32_t)y);
      x = x * s % bb::P;
      y = y * si2 % bb::P;
    }
  }
  auto up = [](uint32_t** d, const std::vector<uint32_t>& h) -> int {
    PLK_HIP(hipMalloc((void**)d, h.size() * 4));
    PLK_HIP(hipMemcpy(*d, h.data(), h.size() * 4, hipMemcpyHostToDevice));
    return PLK_OK;
  };
  {
    // F29 tables, same layouts (root of order 2^26; hi holds 2^14 entries)
    const uint32_t w26 = f29::hpow(f29::GENERATOR, (f29::P - 1) >> f29::TWO_ADICITY);
    const uint32_t w26i = f29::hpow(w26, f29::P - 2);
    std::vector<uint32_t> sf2(SM), si2(SM), lf2(4096), hf2(1 << 14), li2(4096), hi2(1 << 14);
    sf2[0] = si2[0] = f29::to_mont(1);
    for (int j = 0; (1 << j) < SM; j++) {
      const uint32_t wf = f29::hpow(w26, 1ull << (25 - j));   // order 2^(j+1)
      const uint32_t wi = f29::hpow(w26i, 1ull << (25 - j));
      uint64_t xf = 1, xi = 1;
      for (int r = 0; r < (1 << j); r++) {
        sf2[(1 << j) + r] = f29::to_mont((uint32_t)xf);
        si2[(1 << j) + r] = f29::to_mont((uint32_t)xi);
        xf = xf * wf % f29::P;
        xi = xi * wi % f29::P;
      }
    }
    uint64_t x = 1, y = 1;
    for (int i = 0; i < 4096; i++) {
      lf2[i] = f29::to_mont((uint32_t)x);
      li2[i] = f29::to_mont((uint32_t)y);
      x = x * w26 % f29::P;
      y = y * w26i % f29::P;
    }
    const uint64_t st4 = f29::hpow(w26, 4096), st4i = f29::hpow(w26i, 4096);
    x = 1, y = 1;
    for (int i = 0; i < (1 << 14); i++) {
      hf2[i] = f29::to_mont((uint32_t)x);
      hi2[i] = f29::to_mont((uint32_t)y);
      x = x * st4 % f29::P;
      y = y * st4i % f29::P;
    }
    int rc2;
    if ((rc2 = up(&T29.d_small_f, sf2)) || (rc2 = up(&T29.d_small_i, si2)) || (rc2 = up(&T29.d_lo_f, lf2)) ||
        (rc2 = up(&T29.d_hi_f, hf2)) || (rc2 = up(&T29.d_lo_i, li2)) || (rc2 = up(&T29.d_hi_i, hi2))) {
      free_tw(T29);
      return rc2;
    }
  }
  uint32_t m17[17];
  for (int v = 0; v < 17; v++) m17[v] = bb::to_mont((uint32_t)v);
  PLK_HIP(hipMemcpyToSymbol(HIP_SYMBOL(c_mont17), m17, sizeof m17));   // (per device: this one)
  TwHost t{};
  int rc;
  if ((rc = up(&t.d_small_f, sf)) || (rc = up(&t.d_small_i, si)) || (rc = up(&t.d_lo_f, lf)) ||
      (rc = up(&t.d_hi_f, hf)) || (rc = up(&t.d_lo_i, li)) || (rc = up(&t.d_hi_i, hi_))) {
    free_tw(t);
    free_tw(T29);
    return rc;
  }
  T = t;   // (the column tables are built from the root tables of this device)
  if ((rc = plk_wave_init_coltabs())) {
    plk_wave_free_coltabs();
    free_tw(T);   // d_small_f marks the device's tables complete: only with its column tables
    free_tw(T29);
    return rc;
  }
  return PLK_OK;
}

// every device's tables (the current device is restored)
void plk_ntt_free_tables(void) {
  const int prev = plk_cur_device();
  for (int d = 0; d < PLK_MAX_DEVICES; d++) {
    DevTw& t = g_tw[d];
    if (!t.bb.d_small_f && !t.f29.d_small_f) continue;
    (void)hipSetDevice(d);
    free_tw(t.bb);
    free_tw(t.f29);
    plk_wave_free_coltabs();
  }
  (void)hipSetDevice(prev);
}

static int log2_ceil(uint64_t v) {
  int k = 0;
  while ((1ull << k) < v) k++;
  return k;
}

// NTT size of a product.  A result just above a power of two (la + lb - 1 = 2^K + e, e small,
// as every prover shape n+2, 2n+3, 4n+6 at n = 2^m is) is WRAPPED: the full operands go
// through a cyclic transform of 2^K points, so c[2^K + j] (j < e) lands on c[j] (each cyclic
// output still sums at most min(la, lb) terms: exactness bounds unchanged).  Those top e
// coefficients involve only the operands' last e coefficients (e - j terms each): the last
// inverse pass computes them from the bytes and corrects both ends -- half the transform
// size for O(e^2) MACs.
constexpr uint64_t PLK_WRAP_MAX = 16;
static int product_plan(uint64_t la, uint64_t lb, uint64_t* e_out) {
  const uint64_t rl = la + lb - 1;
  int k = log2_ceil(rl);
  uint64_t e = 0;
  const uint64_t lg = la > lb ? la : lb;
  if (k - 1 > PLK_SMALL_LOG) {
    const uint64_t ex = rl - (1ull << (k - 1));
    if (ex <= PLK_WRAP_MAX && ex < lg) { e = ex; k -= 1; }
  }
  if (e_out) *e_out = e;
  return k;
}

// a product that goes through the transform engine (so it can be a sum-group member)
bool plk_poly_mul_summable(uint64_t la, uint64_t lb) {
  const uint64_t mn = la < lb ? la : lb;
  return la && lb && mn > PLK_DIRECT_MAX && product_plan(la, lb, nullptr) > PLK_SMALL_LOG;
}

// Products outside one transform's exact range (min(la, lb) * 256 >= the BabyBear prime, i.e.
// min >= 7,864,320, or a transform above 2^27 points) -- sizes the reference computes with its
// schoolbook loop -- run BLOCKED: the longer operand in pieces of PLK_BLK_L, the shorter in
// pieces of PLK_BLK_S coefficients, every piece product an in-range F29 product of a 2^26-point
// transform, accumulated mod 17 into the zeroed output at the pieces' offset sum.
// PLK_OPT_POLY_BLOCK_L / _S force the blocked path with smaller pieces (tests).
struct BlkSizes {
  uint64_t L, S;   // piece lengths of the longer / shorter operand
  bool forced;
};
static BlkSizes blk_sizes() {
  const int64_t l = plk_opt(PLK_OPT_POLY_BLOCK_L), s = plk_opt(PLK_OPT_POLY_BLOCK_S);
  const bool forced = l >= 33 && s >= 33;
  return forced ? BlkSizes{(uint64_t)l, (uint64_t)s, true}
                : BlkSizes{(1ull << 26) - 3670016 + 1, 3670016, false};   // F29's range: 128 S < p; L + S - 1 = 2^26
}
static bool blocked_shape(uint64_t la, uint64_t lb) {
  const BlkSizes bs = blk_sizes();
  const uint64_t mn = la < lb ? la : lb, mx = la < lb ? lb : la;
  if (bs.forced) return mn > bs.S || mx > bs.L;
  return mn * 256 >= bb::P || product_plan(la, lb, nullptr) > bb::TWO_ADICITY;
}
static size_t blocked_ws(uint64_t la, uint64_t lb);

// direct convolution + trim_kernel: both only plain-store their outputs (no atomics), so their
// operands and outputs may live in mapped host memory (the host ABI's toy-size calls)
bool plk_poly_mul_is_direct(uint64_t la, uint64_t lb) {
  return la && lb && (la < lb ? la : lb) <= PLK_DIRECT_MAX && !blocked_shape(la, lb);
}

size_t plk_poly_mul_workspace_bytes(uint64_t la, uint64_t lb) {
  if (la == 0 || lb == 0) return 0;
  if (blocked_shape(la, lb)) return blocked_ws(la, lb);
  const int k = product_plan(la, lb, nullptr);
  if ((la < lb ? la : lb) <= PLK_DIRECT_MAX || k <= PLK_SMALL_LOG) return 0;
  return (size_t)2 * 4 * (1ull << k);
}

static size_t pass_lds(int M, int C, bool center) {
  const size_t rows = 1u << M;
  return (center ? 2 : 1) * C * (size_t)col_stride((int)rows) * 4 + (center ? 2 : 1) * rows * 4 + (size_t)C * M * 4;
}

// m products of one transform size 2^k through the wave engine (workspace 2^(k+3) bytes each);
// es[i] > 0: a wrapped product (product_plan) with es[i] top coefficients.
// d_nz (single products only): the trimmed length, computed by the last inverse pass
static int ntt_group(const PlkPolyMulJob* g, int m, int k, const uint64_t* es, void* d_work, hipStream_t st,
                     uint32_t* d_nz = nullptr) {
  PLK_MARK(3);
  // F29 (lazy reduction, fewer VALU per butterfly) whenever every convolution term fits it
  bool use29 = plk_opt(PLK_OPT_NTT_F29) && k <= f29::TWO_ADICITY;
  for (int i = 0; i < m; i++) {
    // a sum group must fit as a whole: 64 sum(min(la, lb)) <= (p - 1) / 2
    uint64_t mn = 0;
    int gs = 0;
    do {
      mn += g[i + gs].la < g[i + gs].lb ? g[i + gs].la : g[i + gs].lb;
      gs++;
    } while (i + gs < m && g[i + gs].acc);
    if (mn * 128 >= f29::P) use29 = false;   // centered residues (F29::byte_val)
    if (!use29 && mn * 256 >= bb::P) {
      plk_set_error("poly_mul batch: a sum of %d products of %llu coefficients in all exceeds both fields", gs,
                    (unsigned long long)mn);
      return PLK_ERR_RANGE;
    }
  }
  // final scale: the transform's inputs are normal-form byte values (not Montgomery), so the
  // Montgomery pointwise product leaves a factor R^-1: N^-1 R^2, applied by one more Montgomery
  // multiply, gives the normal-form coefficient
  const uint32_t ninv = use29 ? (uint32_t)((uint64_t)f29::hpow(1ull << k, f29::P - 2) * f29::R2 % f29::P)
                              : (uint32_t)((uint64_t)bb::hpow(1ull << k, bb::P - 2) * bb::R2 % bb::P);
  // operands: job i owns slots 2i (a) and 2i+1 (b) of d_work; an operand equal (same bytes,
  // same length) to an earlier one of the same launch chunk (PLK_WAVE_MAX_JOBS jobs: a chunk's
  // forward passes transform its distinct arrays) reuses that slot's transform
  const bool noshare = !plk_opt(PLK_OPT_NTT_SHARE);
  uint32_t* W = (uint32_t*)d_work;
  int slot[64][2], refs[128] = {0};
  bool fixb[64];   // b's forward transform supplied (PlkPolyMulJob::bt) for this k and field
  for (int i = 0; i < m; i++) fixb[i] = g[i].bt && g[i].bt_k == k && g[i].bt_field == (use29 ? 1 : 0);
  for (int i = 0; i < m; i++)
    for (int s = 0; s < 2; s++) {
      if (s && fixb[i]) {
        slot[i][1] = -1;
        continue;
      }
      const uint8_t* ptr = s ? g[i].b : g[i].a;
      const uint64_t len = s ? g[i].lb : g[i].la;
      slot[i][s] = 2 * i + s;
      for (int q = i - i % PLK_WAVE_MAX_JOBS; q <= i && !noshare; q++)
        for (int t = 0; t < 2 && (q < i || t < s); t++)
          if ((t ? g[q].b : g[q].a) == ptr && (t ? g[q].lb : g[q].la) == len && slot[q][t] == 2 * q + t) {
            slot[i][s] = 2 * q + t;
            q = i + 1;
            break;
          }
      refs[slot[i][s]]++;
    }
  // the center output of job i goes to an operand slot only job i reads, else to a free slot
  int cslot[64], nfree = 0, freel[128];
  for (int x = 0; x < 2 * m; x++)
    if (!refs[x]) freel[nfree++] = x;
  for (int i = 0; i < m; i++) {
    cslot[i] = -1;
    for (int s = 0; s < 2 && cslot[i] < 0; s++)
      if (slot[i][s] == 2 * i + s && refs[2 * i + s] == 1) cslot[i] = 2 * i + s;
    if (cslot[i] < 0) {
      if (!nfree) {   // (cannot happen: every shared reference leaves a slot unused)
        plk_set_error("poly_mul batch: no free work array for job %d", i);
        return PLK_ERR_ARG;
      }
      cslot[i] = freel[--nfree];
    }
  }
  WJob w[64];
  for (int i = 0; i < m; i++) {
    const PlkPolyMulJob& j = g[i];
    const uint64_t e = es ? es[i] : 0;
    // (a supplied b transform has no slot: B is the caller's words, read only)
    uint32_t* B = fixb[i] ? const_cast<uint32_t*>(j.bt) : W + ((size_t)slot[i][1] << k);
    w[i] = WJob{j.a, j.b, j.la, j.lb, j.out, j.la + j.lb - 1 - e, W + ((size_t)slot[i][0] << k), B,
                W + ((size_t)cslot[i] << k)};
    w[i].ntop = (int)e;
    w[i].bfix = fixb[i] ? 1 : 0;
    w[i].der = j.der;
  }
  if (m == 1) w[0].nz = d_nz;
  // sum groups: a member (acc) adds its center output into its leader's first inverse pass
  for (int i = 0, L = 0; i < m; i++) {
    if (!g[i].acc) {
      L = i;
      continue;
    }
    // (one transform size, checked by the caller; no member longer than the leader's product,
    // so its wrapped top, if any, is within the leader's)
    if (i == 0 || g[i].la + g[i].lb > g[L].la + g[L].lb || w[L].ngroup == 2 ||
        L / PLK_WAVE_MAX_JOBS != i / PLK_WAVE_MAX_JOBS) {   // (a group runs in one launch chunk)
      plk_set_error("poly_mul batch: invalid sum group at job %d", i);
      return PLK_ERR_ARG;
    }
    (w[L].ngroup ? w[L].S2 : w[L].S1) = w[i].C;
    w[L].ga8[w[L].ngroup] = w[i].a8;
    w[L].gla[w[L].ngroup] = w[i].la;
    w[L].glb[w[L].ngroup] = w[i].lb;
    w[L].gb8[w[L].ngroup++] = w[i].b8;
    w[i].skip_inv = 1;
  }
  return plk_wave_poly_mul_batch_launch(w, m, k, use29 ? 1 : 0, ninv, st);
}

// out[off + t] = (out[off + t] + part[t]) mod 17, t < len (a piece product of the blocked path)
__global__ __launch_bounds__(256) void acc17_kernel(uint8_t* __restrict__ out, const uint8_t* __restrict__ part,
                                                    uint64_t len) {
  for (uint64_t t = (uint64_t)blockIdx.x * 256 + threadIdx.x; t < len; t += (uint64_t)gridDim.x * 256)
    out[t] = (uint8_t)((out[t] + part[t]) % 17u);
}

static uint64_t align256(uint64_t v) { return (v + 255) & ~255ull; }
// workspace of the blocked path: one piece product's bytes + the largest piece's own workspace
static size_t blocked_ws(uint64_t la, uint64_t lb) {
  const BlkSizes bs = blk_sizes();
  const uint64_t mn = la < lb ? la : lb, mx = la < lb ? lb : la;
  const uint64_t pl = mx < bs.L ? mx : bs.L, ps = mn < bs.S ? mn : bs.S;
  return (size_t)align256(pl + ps - 1) + plk_poly_mul_workspace_bytes(pl, ps);
}

int plk_poly_mul_launch(const uint8_t* d_a, uint64_t la, const uint8_t* d_b, uint64_t lb, uint8_t* d_out,
                        uint32_t* d_nz, void* d_work, hipStream_t st);
static int blocked_launch(const uint8_t* d_a, uint64_t la, const uint8_t* d_b, uint64_t lb, uint8_t* d_out,
                          uint32_t* d_nz, void* d_work, hipStream_t st) {
  if (!d_work) {
    plk_set_error("poly_mul: %llu x %llu needs a workspace (plk_poly_mul_workspace)", (unsigned long long)la,
                  (unsigned long long)lb);
    return PLK_ERR_ARG;
  }
  const bool aL = la >= lb;
  const uint8_t* L = aL ? d_a : d_b;
  const uint8_t* S = aL ? d_b : d_a;
  const uint64_t lL = aL ? la : lb, lS = aL ? lb : la, rl = la + lb - 1;
  const BlkSizes bs = blk_sizes();
  const uint64_t pl = lL < bs.L ? lL : bs.L, ps = lS < bs.S ? lS : bs.S;
  uint8_t* part = (uint8_t*)d_work;
  void* pwork = part + align256(pl + ps - 1);
  PLK_HIP(hipMemsetAsync(d_out, 0, rl, st));
  for (uint64_t i = 0; i < lL; i += bs.L)
    for (uint64_t j = 0; j < lS; j += bs.S) {
      const uint64_t li = lL - i < bs.L ? lL - i : bs.L, lj = lS - j < bs.S ? lS - j : bs.S;
      int rc = plk_poly_mul_launch(L + i, li, S + j, lj, part, nullptr, pwork, st);
      if (rc) return rc;
      const uint64_t len = li + lj - 1, blocks = (len + 255) / 256;
      hipLaunchKernelGGL(acc17_kernel, dim3((unsigned)(blocks < 16384 ? blocks : 16384)), dim3(256), 0, st,
                         d_out + i + j, part, len);
      PLK_HIP(hipGetLastError());
    }
  if (d_nz) hipLaunchKernelGGL(trim_kernel, dim3(1), dim3(1024), 0, st, d_out, rl, d_nz);
  PLK_HIP(hipGetLastError());
  return PLK_OK;
}

// d_out must hold la+lb-1 bytes; *d_nz (if not NULL) receives the trimmed length (0 means "all zero" ->
// the caller reports length 1).
int plk_poly_mul_launch(const uint8_t* d_a, uint64_t la, const uint8_t* d_b, uint64_t lb, uint8_t* d_out,
                        uint32_t* d_nz, void* d_work, hipStream_t st) {
  if (la == 0 || lb == 0) {
    plk_set_error("poly_mul: empty operand (la %llu, lb %llu)", (unsigned long long)la, (unsigned long long)lb);
    return PLK_ERR_ARG;
  }
  const uint64_t rl = la + lb - 1;
  const uint64_t mn = la < lb ? la : lb;
  if (rl >= (1ull << 32)) {   // (the trimmed length is a 32-bit word)
    plk_set_error("poly_mul: %llu x %llu: la + lb - 1 must be < 2^32", (unsigned long long)la,
                  (unsigned long long)lb);
    return PLK_ERR_RANGE;
  }
  if (blocked_shape(la, lb)) return blocked_launch(d_a, la, d_b, lb, d_out, d_nz, d_work, st);
  if (mn <= PLK_DIRECT_MAX) {
    const uint8_t* lg = la >= lb ? d_a : d_b;
    const uint8_t* sh = la >= lb ? d_b : d_a;
    const uint64_t blocks64 = (rl + 255) / 256;
    const int blocks = (int)(blocks64 > 8192 ? 8192 : blocks64);
    hipLaunchKernelGGL(polymul_direct_kernel, dim3(blocks), dim3(256), 0, st, lg, la >= lb ? la : lb, sh, (int)mn,
                       d_out, d_nz);
    PLK_HIP(hipGetLastError());
    if (d_nz) hipLaunchKernelGGL(trim_kernel, dim3(1), dim3(1024), 0, st, d_out, rl, d_nz);
    PLK_HIP(hipGetLastError());
    return PLK_OK;
  }
  uint64_t e = 0;
  const int k = product_plan(la, lb, &e);
  if (k > bb::TWO_ADICITY) {
    plk_set_error("poly_mul: %llu x %llu needs a 2^%d transform (max 2^%d)", (unsigned long long)la,
                  (unsigned long long)lb, k, bb::TWO_ADICITY);
    return PLK_ERR_RANGE;
  }
  const uint32_t ninv = bb::hpow(1ull << k, bb::P - 2);   // normal form on purpose
  if (k <= PLK_SMALL_LOG) {   // (never wrapped: product_plan only wraps above 2^(SMALL_LOG+1))
    const size_t lds = (size_t)4 * (2 * col_stride(1 << k) + 2 * (1 << k));
    hipLaunchKernelGGL(polymul_small_kernel, dim3(1), dim3(1024), lds, st, d_a, la, d_b, lb, k, tw_fwd(), tw_inv(),
                       d_out, ninv, d_nz);
    PLK_HIP(hipGetLastError());
    return PLK_OK;
  }
  if (!d_work) {
    plk_set_error("poly_mul: %llu x %llu needs a workspace (plk_poly_mul_workspace)", (unsigned long long)la,
                  (unsigned long long)lb);
    return PLK_ERR_ARG;
  }
  const PlkPolyMulJob job{d_a, la, d_b, lb, d_out};
  // (the trimmed length comes out of the last inverse pass: no trim_kernel launch)
  return ntt_group(&job, 1, k, e ? &e : nullptr, d_work, st, d_nz);
}

int plk_poly_mul_transform_plan(uint64_t la, uint64_t lb, int* field) {
  if (!la || !lb || blocked_shape(la, lb)) return -1;
  const uint64_t mn = la < lb ? la : lb;
  const int k = product_plan(la, lb, nullptr);
  if (mn <= PLK_DIRECT_MAX || k <= PLK_SMALL_LOG || !plk_wave_ntt_supported(k)) return -1;
  const bool use29 = plk_opt(PLK_OPT_NTT_F29) && k <= f29::TWO_ADICITY && mn * 128 < f29::P;
  if (field) *field = use29 ? 1 : 0;
  return k;
}

int plk_poly_mul_pretransform(const uint8_t* d_b, uint64_t lb, int k, int field, uint32_t* d_out, hipStream_t st) {
  if (field == 1 && k > f29::TWO_ADICITY) {
    plk_set_error("pretransform: 2^%d is beyond F29's roots", k);
    return PLK_ERR_RANGE;
  }
  return plk_wave_pretransform(d_b, lb, k, field, d_out, st);
}

// Several independent products: direct / one-workgroup ones one by one, the NTT ones grouped
// by transform size and run as batches through the wave engine (one launch per pass for the
// whole group; job i of a group uses 2^(k+3) bytes of d_work at offset i 2^(k+3)).  The
// prover's round-3 products come in such groups (7 at 2^21, then 3 + 2 at 2^22 for n = 2^20).
int plk_poly_mul_batch_launch(const PlkPolyMulJob* jobs, int nj, void* d_work, size_t work_bytes, hipStream_t st) {
  PLK_MARK(2);
  int ks[64];
  uint64_t es[64];
  if (nj > 64) {
    plk_set_error("poly_mul batch of %d products (max 64)", nj);
    return PLK_ERR_RANGE;
  }
  for (int i = 0; i < nj; i++) {
    const PlkPolyMulJob& j = jobs[i];
    ks[i] = -1;
    if (j.la == 0 || j.lb == 0) {
      plk_set_error("poly_mul batch: job %d has an empty operand", i);
      return PLK_ERR_ARG;
    }
    const uint64_t mn = j.la < j.lb ? j.la : j.lb;
    const int k = product_plan(j.la, j.lb, &es[i]);
    if (j.acc && !(mn > PLK_DIRECT_MAX && k > PLK_SMALL_LOG)) {
      plk_set_error("poly_mul batch: sum-group member %d is not a transform-sized product", i);
      return PLK_ERR_ARG;
    }
    if (j.acc) {   // adds into the group's leader: the last non-member before it
      int L = i - 1;
      while (L > 0 && jobs[L].acc) L--;
      if (i == 0 || jobs[L].acc || ks[L] != k || j.la + j.lb > jobs[L].la + jobs[L].lb) {
        plk_set_error("poly_mul batch: sum-group member %d does not follow a product of its transform size and at "
                      "least its length", i);
        return PLK_ERR_ARG;
      }
    }
    if (mn > PLK_DIRECT_MAX && k > PLK_SMALL_LOG) {
      if (mn * 256 >= bb::P || k > bb::TWO_ADICITY) {
        plk_set_error("poly_mul batch: job %d (%llu x %llu) outside the exact range", i, (unsigned long long)j.la,
                      (unsigned long long)j.lb);
        return PLK_ERR_RANGE;
      }
      ks[i] = k;
      continue;
    }
    if (j.der) {   // (the derived bytes come from the wave engine's first forward pass)
      plk_set_error("poly_mul batch: job %d derives its operand but is not a transform-sized product", i);
      return PLK_ERR_ARG;
    }
    const int rc = plk_poly_mul_launch(j.a, j.la, j.b, j.lb, j.out, nullptr, nullptr, st);
    if (rc) return rc;
  }
  bool done[64] = {false};
  for (int i = 0; i < nj; i++) {
    if (ks[i] < 0 || done[i]) continue;
    const int k = ks[i];
    const size_t per = (size_t)8 << k;
    // a sub-group fits the workspace and one launch chunk of the wave engine, and never splits
    // a sum group (a leader and the acc members right after it)
    const size_t fit = work_bytes / per;
    const int cap = (int)(fit < (size_t)PLK_WAVE_MAX_JOBS ? fit : (size_t)PLK_WAVE_MAX_JOBS);
    if (cap < 1) {
      plk_set_error("poly_mul batch: workspace %zu bytes < %zu", work_bytes, per);
      return PLK_ERR_ARG;
    }
    PlkPolyMulJob g[64];
    uint64_t ge[64];
    int m = 0;
    for (int q = i; q < nj; q++) {
      if (done[q] || ks[q] != k || jobs[q].acc) continue;   // (members come with their leader)
      int gs = 1;
      while (q + gs < nj && jobs[q + gs].acc) gs++;
      if (m + gs > cap) {
        if (m == 0) {
          plk_set_error("poly_mul batch: a sum group of %d products needs %zu workspace bytes", gs, per * gs);
          return PLK_ERR_ARG;
        }
        break;
      }
      for (int u = 0; u < gs; u++) {
        g[m] = jobs[q + u];
        ge[m++] = es[q + u];
        done[q + u] = true;
      }
    }
    const int rc = ntt_group(g, m, k, ge, d_work, st);
    if (rc) return rc;
  }
  return PLK_OK;
}

// Standalone forward NTT (DIF, natural -> bit-reversed), in place on Montgomery-form u32,
// or inverse (DIT, bit-reversed -> natural, NOT scaled by N^-1).  Same passes as poly_mul.
// batch independent arrays at d + b 2^k share each pass's launch (up to 12 per launch).
// F29 (p = 7 2^26 + 1, the field poly_mul and the prover transform in): the wave engine only,
// 2^13 .. 2^26 points, results fully reduced
int plk_ntt29_launch(uint32_t* d, int k, int batch, int inverse, hipStream_t st) {
  if (k < 13 || k > f29::TWO_ADICITY || batch < 1) {
    plk_set_error("ntt29: log_n %d (13..%d), batch %d", k, f29::TWO_ADICITY, batch);
    return PLK_ERR_RANGE;
  }
  return plk_wave_ntt_launch(d, k, batch, inverse, 1, st);
}

int plk_ntt_launch(uint32_t* d, int k, int batch, int inverse, hipStream_t st) {
  if (k < 1 || k > bb::TWO_ADICITY || batch < 1) {
    plk_set_error("ntt: log_n %d (1..%d), batch %d", k, bb::TWO_ADICITY, batch);
    return PLK_ERR_RANGE;
  }
  if (plk_wave_ntt_supported(k)) return plk_wave_ntt_launch(d, k, batch, inverse, 0, st);
  // k <= 12: one workgroup-tile pass (lo = 0, a single tile holds the whole array)
  const Tw tw = inverse ? tw_inv() : tw_fwd();
  const Pass p{k, 0, k, 1};
  const size_t lds = pass_lds(p.M, p.C, false);
  for (int b = 0; b < batch; b++) {
    uint32_t* db = d + ((uint64_t)b << k);
    if (inverse)
      hipLaunchKernelGGL((ntt_pass_kernel<true, IN_U32, OUT_U32>), dim3(1, 1), dim3(NTT_THREADS), lds, st, p, db, db,
                         nullptr, nullptr, 0, 0, tw, nullptr, 0, 0u, nullptr);
    else
      hipLaunchKernelGGL((ntt_pass_kernel<false, IN_U32, OUT_U32>), dim3(1, 1), dim3(NTT_THREADS), lds, st, p, db, db,
                         nullptr, nullptr, 0, 0, tw, nullptr, 0, 0u, nullptr);
  }
  PLK_HIP(hipGetLastError());
  return PLK_OK;
}
