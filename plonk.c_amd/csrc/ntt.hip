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

// max over the block (blockDim a multiple of 64, <= 1024); every thread gets the result
__device__ __forceinline__ uint32_t block_max(uint32_t v) {
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
  last = block_max(last);
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
    last = block_max(last);
    if (last) {
      if (threadIdx.x == 0) *nz = last;
      return;
    }
  }
  if (threadIdx.x == 0) *nz = 0;
}

// Direct convolution when one operand is short: out[i] = sum_j a[j] b[i-j] mod 17 over the
// short operand s (length ls <= 32, staged in LDS), the long one read coalesced.
__global__ __launch_bounds__(256) void polymul_direct_kernel(const uint8_t* lg, uint64_t llg, const uint8_t* sh,
                                                             int lsh, uint8_t* out8, uint32_t* nz) {
  __shared__ uint32_t S[64];
  if (threadIdx.x < lsh) S[threadIdx.x] = sh[threadIdx.x] % 17u;
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

// Batched tails of split products (one launch for a whole product group, blockIdx.y = job):
// out[i] += sum_{j < lt} t[j] g[i - base - j] for i in [base, rl), out[i] for i >= ntt_len not
// yet written (taken as 0).  16 outputs per thread, chunks aligned to the OUTPUT (one uint4
// read-modify-write); the 32-byte g window is funnel-shifted out of three aligned uint4 loads
// and each output is four v_dot4_u32_u8 of the reversed t against the window's bytes.
struct TailJob {
  const uint8_t* g;
  uint64_t lg;
  const uint8_t* t;
  int lt;           // <= 16
  uint64_t base, ntt_len, rl;
  uint8_t* out8;
  // a sum group's members: the same shape, their own g and t added into the same outputs
  const uint8_t* g2[2];
  const uint8_t* t2[2];
};
constexpr int TAIL_MAX_JOBS = 12;
struct TailJobs {
  TailJob j[TAIL_MAX_JOBS];
};

__device__ __forceinline__ uint32_t mod17_small(uint32_t a) {   // a < 2^13
  const uint32_t q = (a * 61681u) >> 20;
  return a - 17u * q;
}
// any byte of x above 16 (false positives only next to bytes >= 0x80)
__device__ __forceinline__ bool bytes_over16(uint32_t x) { return (((x + 0x6F6F6F6Fu) | x) & 0x80808080u) != 0; }
__device__ __forceinline__ uint32_t bytes_mod17(uint32_t x) {
  uint32_t r = 0;
#pragma unroll
  for (int b = 0; b < 4; b++) r |= (((x >> (8 * b)) & 0xFFu) % 17u) << (8 * b);
  return r;
}

// 16 outputs' tail sums of one (g, t) pair, added into acc (bytes in packed words)
__device__ __forceinline__ void tail_pair(const uint8_t* g, uint64_t lg, const uint8_t* t, int lt, int64_t o0,
                                          int64_t s, bool galign, uint32_t (&acc)[16]) {
  uint32_t Tr[4] = {0, 0, 0, 0};   // byte j' = t[15 - j'] mod 17
#pragma unroll
  for (int j = 0; j < 16; j++) {
    const uint32_t v = j < lt ? t[j] % 17u : 0u;
    Tr[(15 - j) >> 2] |= v << (8 * ((15 - j) & 3));
  }
  const int64_t ws = o0 - 15;                        // window bytes g[ws + q], q < 32
  uint32_t W[8];
  const int64_t A = ws - s;                          // 16-byte aligned
  if (galign && A >= 0 && (uint64_t)(A + 48) <= lg) {
    uint32_t L[12];
#pragma unroll
    for (int v = 0; v < 3; v++) {
      const uint4 q = *reinterpret_cast<const uint4*>(g + A + 16 * v);
      L[4 * v] = q.x; L[4 * v + 1] = q.y; L[4 * v + 2] = q.z; L[4 * v + 3] = q.w;
    }
    const uint32_t r = (uint32_t)(s & 3);
    switch (s >> 2) {   // uniform
#define PLK_TAIL_W(Q)                                                                          \
  case Q:                                                                                     \
    _Pragma("unroll") for (int m = 0; m < 8; m++) W[m] = __builtin_amdgcn_alignbyte(L[Q + m + 1], L[Q + m], r); \
    break;
      PLK_TAIL_W(0) PLK_TAIL_W(1) PLK_TAIL_W(2) PLK_TAIL_W(3)
#undef PLK_TAIL_W
    }
  } else {
#pragma unroll
    for (int m = 0; m < 8; m++) {
      uint32_t w = 0;
#pragma unroll
      for (int b = 0; b < 4; b++) {
        const int64_t o = ws + 4 * m + b;
        if (o >= 0 && (uint64_t)o < lg) w |= (uint32_t)g[o] << (8 * b);
      }
      W[m] = w;
    }
  }
  bool big = false;
#pragma unroll
  for (int m = 0; m < 8; m++) big |= bytes_over16(W[m]);
  if (big) {
#pragma unroll
    for (int m = 0; m < 8; m++) W[m] = bytes_mod17(W[m]);
  }
#pragma unroll
  for (int k = 0; k < 16; k++) {
#pragma unroll
    for (int m = 0; m < 4; m++) {
      const int i = (k >> 2) + m;
      const uint32_t wd = (k & 3) ? __builtin_amdgcn_alignbyte(W[i + 1], W[i], k & 3) : W[i];
      acc[k] = __builtin_amdgcn_udot4(Tr[m], wd, acc[k], false);
    }
  }
}

__global__ __launch_bounds__(256) void polymul_tail_batch_kernel(TailJobs J) {
  const TailJob& jb = J.j[blockIdx.y];
  const uint64_t span = jb.rl - jb.base;
  uint8_t* const ob = jb.out8 + jb.base;
  const int64_t d = (int64_t)((uintptr_t)ob & 15);     // chunk c: outputs o in [16c - d, 16c - d + 16)
  const int64_t s = (int64_t)((1 - d) & 15);           // window start mod 16
  for (uint64_t c = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; 16 * c < span + d;
       c += (uint64_t)gridDim.x * blockDim.x) {
    const int64_t o0 = (int64_t)(16 * c) - d;
    // current outputs (0 where not yet written by the transform)
    uint32_t acc[16];
    const bool full = o0 >= 0 && (uint64_t)(o0 + 16) <= span;
    if (full && jb.base + (uint64_t)o0 + 16 <= jb.ntt_len) {
      const uint4 q = *reinterpret_cast<const uint4*>(ob + o0);
      const uint32_t cur[4] = {q.x, q.y, q.z, q.w};
#pragma unroll
      for (int k = 0; k < 16; k++) acc[k] = (cur[k >> 2] >> (8 * (k & 3))) & 0xFFu;
    } else {
#pragma unroll
      for (int k = 0; k < 16; k++) {
        const int64_t o = o0 + k;
        acc[k] = (o >= 0 && (uint64_t)o < span && jb.base + (uint64_t)o < jb.ntt_len) ? ob[o] : 0u;
      }
    }
    tail_pair(jb.g, jb.lg, jb.t, jb.lt, o0, s, ((uintptr_t)jb.g & 15) == 0, acc);
#pragma unroll
    for (int q = 0; q < 2; q++)
      if (jb.g2[q]) tail_pair(jb.g2[q], jb.lg, jb.t2[q], jb.lt, o0, s, ((uintptr_t)jb.g2[q] & 15) == 0, acc);
    uint32_t res[4] = {0, 0, 0, 0};
#pragma unroll
    for (int k = 0; k < 16; k++) res[k >> 2] |= mod17_small(acc[k]) << (8 * (k & 3));
    if (full) {
      *reinterpret_cast<uint4*>(ob + o0) = make_uint4(res[0], res[1], res[2], res[3]);
    } else {
#pragma unroll
      for (int k = 0; k < 16; k++) {
        const int64_t o = o0 + k;
        if (o >= 0 && (uint64_t)o < span) ob[o] = (uint8_t)(res[k >> 2] >> (8 * (k & 3)));
      }
    }
  }
}

// ------------------------------------------------------------------------------ host side
namespace {

struct TwHost {
  uint32_t* d_small_f = nullptr;
  uint32_t* d_small_i = nullptr;
  uint32_t* d_lo_f = nullptr;
  uint32_t* d_hi_f = nullptr;
  uint32_t* d_lo_i = nullptr;
  uint32_t* d_hi_i = nullptr;
} g_tw;

Tw tw_fwd() { return Tw{g_tw.d_small_f, g_tw.d_lo_f, g_tw.d_hi_f}; }
Tw tw_inv() { return Tw{g_tw.d_small_i, g_tw.d_lo_i, g_tw.d_hi_i}; }

}  // namespace

static struct {
  uint32_t *d_small_f = nullptr, *d_small_i = nullptr, *d_lo_f = nullptr, *d_hi_f = nullptr, *d_lo_i = nullptr,
           *d_hi_i = nullptr;
} g_tw29;

PlkTwTables plk_ntt_tables29(void) {
  return PlkTwTables{g_tw29.d_small_f, g_tw29.d_small_i, g_tw29.d_lo_f, g_tw29.d_hi_f, g_tw29.d_lo_i, g_tw29.d_hi_i};
}

PlkTwTables plk_ntt_tables(void) {
  return PlkTwTables{g_tw.d_small_f, g_tw.d_small_i, g_tw.d_lo_f, g_tw.d_hi_f, g_tw.d_lo_i, g_tw.d_hi_i};
}

int plk_ntt_init_tables(void) {
  if (g_tw.d_small_f) return PLK_OK;
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
    auto up2 = [](uint32_t** d, const std::vector<uint32_t>& h) -> int {
      PLK_HIP(hipMalloc((void**)d, h.size() * 4));
      PLK_HIP(hipMemcpy(*d, h.data(), h.size() * 4, hipMemcpyHostToDevice));
      return PLK_OK;
    };
    int rc2;
    if ((rc2 = up2(&g_tw29.d_small_f, sf2)) || (rc2 = up2(&g_tw29.d_small_i, si2)) || (rc2 = up2(&g_tw29.d_lo_f, lf2)) ||
        (rc2 = up2(&g_tw29.d_hi_f, hf2)) || (rc2 = up2(&g_tw29.d_lo_i, li2)) || (rc2 = up2(&g_tw29.d_hi_i, hi2)))
      return rc2;
  }
  uint32_t m17[17];
  for (int v = 0; v < 17; v++) m17[v] = bb::to_mont((uint32_t)v);
  PLK_HIP(hipMemcpyToSymbol(HIP_SYMBOL(c_mont17), m17, sizeof m17));
  auto up = [](uint32_t** d, const std::vector<uint32_t>& h) -> int {
    PLK_HIP(hipMalloc((void**)d, h.size() * 4));
    PLK_HIP(hipMemcpy(*d, h.data(), h.size() * 4, hipMemcpyHostToDevice));
    return PLK_OK;
  };
  int rc;
  if ((rc = up(&g_tw.d_small_f, sf)) || (rc = up(&g_tw.d_small_i, si)) || (rc = up(&g_tw.d_lo_f, lf)) ||
      (rc = up(&g_tw.d_hi_f, hf)) || (rc = up(&g_tw.d_lo_i, li)) || (rc = up(&g_tw.d_hi_i, hi_)))
    return rc;
  return plk_wave_init_coltabs();
}

void plk_ntt_free_tables(void) {
  (void)hipFree(g_tw.d_small_f); (void)hipFree(g_tw.d_small_i); (void)hipFree(g_tw.d_lo_f);
  (void)hipFree(g_tw.d_hi_f); (void)hipFree(g_tw.d_lo_i); (void)hipFree(g_tw.d_hi_i);
  (void)hipFree(g_tw29.d_small_f); (void)hipFree(g_tw29.d_small_i); (void)hipFree(g_tw29.d_lo_f);
  (void)hipFree(g_tw29.d_hi_f); (void)hipFree(g_tw29.d_lo_i); (void)hipFree(g_tw29.d_hi_i);
  g_tw29.d_small_f = g_tw29.d_small_i = g_tw29.d_lo_f = g_tw29.d_hi_f = g_tw29.d_lo_i = g_tw29.d_hi_i = nullptr;
  g_tw = TwHost{};
  plk_wave_free_coltabs();
}

static int log2_ceil(uint64_t v) {
  int k = 0;
  while ((1ull << k) < v) k++;
  return k;
}

// NTT size of a product.  A result just above a power of two (la + lb - 1 = 2^K + e, e small,
// as every prover shape n+2, 2n+3, 4n+6 at n = 2^m is) is split: the longer operand's last e
// coefficients t are taken out, the rest times the other operand fills exactly 2^K, and
// x^(la-e) t(x) b(x) is added by polymul_tail_batch_kernel -- half the transform size for O(e n) MACs.
constexpr uint64_t PLK_SPLIT_MAX = 16;
static int product_plan(uint64_t la, uint64_t lb, uint64_t* e_out) {
  const uint64_t rl = la + lb - 1;
  int k = log2_ceil(rl);
  uint64_t e = 0;
  const uint64_t lg = la > lb ? la : lb;
  if (k - 1 > PLK_SMALL_LOG) {
    const uint64_t ex = rl - (1ull << (k - 1));
    if (ex <= PLK_SPLIT_MAX && ex < lg) { e = ex; k -= 1; }
  }
  if (e_out) *e_out = e;
  return k;
}

// a product that goes through the transform engine (so it can be a sum-group member)
bool plk_poly_mul_summable(uint64_t la, uint64_t lb) {
  const uint64_t mn = la < lb ? la : lb;
  return la && lb && mn > PLK_DIRECT_MAX && product_plan(la, lb, nullptr) > PLK_SMALL_LOG;
}

size_t plk_poly_mul_workspace_bytes(uint64_t la, uint64_t lb) {
  if (la == 0 || lb == 0) return 0;
  const int k = product_plan(la, lb, nullptr);
  if ((la < lb ? la : lb) <= PLK_DIRECT_MAX || k <= PLK_SMALL_LOG) return 0;
  return (size_t)2 * 4 * (1ull << k);
}

static size_t pass_lds(int M, int C, bool center) {
  const size_t rows = 1u << M;
  return (center ? 2 : 1) * C * (size_t)col_stride((int)rows) * 4 + (center ? 2 : 1) * rows * 4 + (size_t)C * M * 4;
}

// m products of one transform size 2^k through the wave engine (workspace 2^(k+3) bytes each);
// es[i] > 0: the split plan (product_plan) -- the longer operand's last es[i] coefficients are
// multiplied in directly by polymul_tail_batch_kernel after the transform.
static int ntt_group(const PlkPolyMulJob* g, int m, int k, const uint64_t* es, void* d_work, hipStream_t st) {
  // F29 (lazy reduction, fewer VALU per butterfly) whenever every convolution term fits it
  static int no29 = -1;
  if (no29 < 0) {
    const char* e = getenv("PLK_NTT_NO_F29");
    no29 = e && atoi(e) != 0;
  }
  bool use29 = !no29 && k <= f29::TWO_ADICITY;
  for (int i = 0; i < m; i++) {
    // a sum group of gs products must fit as a whole: gs * 64 min <= (p - 1) / 2
    int gs = 1;
    while (i + gs < m && g[i + gs].acc) gs++;
    const uint64_t mn = g[i].la < g[i].lb ? g[i].la : g[i].lb;
    if ((uint64_t)gs * mn * 128 >= f29::P) use29 = false;   // centered residues (F29::from_byte)
    if (!use29 && (uint64_t)gs * mn * 256 >= bb::P) {
      plk_set_error("poly_mul batch: a sum of %d products of %llu coefficients exceeds both fields", gs,
                    (unsigned long long)mn);
      return PLK_ERR_RANGE;
    }
  }
  const uint32_t ninv = use29 ? f29::hpow(1ull << k, f29::P - 2) : bb::hpow(1ull << k, bb::P - 2);   // normal form
  WJob w[64];
  for (int i = 0; i < m; i++) {
    const PlkPolyMulJob& j = g[i];
    const uint64_t e = es ? es[i] : 0;
    const bool swap = e && j.lb > j.la;                   // a := the longer operand when splitting
    const uint8_t* lgp = swap ? j.b : j.a;
    const uint8_t* shp = swap ? j.a : j.b;
    const uint64_t llg = swap ? j.lb : j.la, lsh = swap ? j.la : j.lb;
    uint32_t* A = (uint32_t*)d_work + ((size_t)2 * i << k);
    w[i] = WJob{lgp, shp, llg - e, lsh, j.out, llg - e + lsh - 1, A, A + (1ull << k)};
  }
  // sum groups: a member (acc) adds its center output into its leader's first inverse pass
  int lead[64];
  for (int i = 0; i < m; i++) {
    lead[i] = i;
    if (!g[i].acc) continue;
    const int L = lead[i - (i > 0)];
    if (i == 0 || g[L].la != g[i].la || g[L].lb != g[i].lb || (es && es[L] != es[i]) || (w[L].S1 && w[L].S2)) {
      plk_set_error("poly_mul batch: invalid sum group at job %d", i);
      return PLK_ERR_ARG;
    }
    lead[i] = L;
    (w[L].S1 ? w[L].S2 : w[L].S1) = w[i].A;
    w[i].skip_inv = 1;
  }
  int rc = plk_wave_poly_mul_batch_launch(w, m, k, use29 ? 1 : 0, ninv, st);
  if (rc) return rc;
  // the tails of the split products (a sum group's in its leader's tail job), one launch per 12
  TailJobs tj{};
  int nt = 0, tj_of[64];
  uint64_t maxspan = 0;
  for (int i = 0; i <= m; i++) {
    if (i < m && es && es[i] && g[i].acc) {
      TailJob& L = tj.j[tj_of[lead[i]]];
      const int q = L.g2[0] ? 1 : 0;
      L.g2[q] = w[i].b8;
      L.t2[q] = w[i].a8 + w[i].la;
      continue;
    }
    // a group's members follow their leader: flush only between groups
    if (i < m && es && es[i]) {
      if (nt == TAIL_MAX_JOBS) {
        const uint64_t blocks64 = (maxspan + 16 * 256 - 1) / (16 * 256);
        hipLaunchKernelGGL(polymul_tail_batch_kernel, dim3((unsigned)std::min<uint64_t>(blocks64, 4096), nt), dim3(256),
                           0, st, tj);
        PLK_HIP(hipGetLastError());
        tj = TailJobs{};
        nt = 0;
        maxspan = 0;
      }
      const uint64_t rl = g[i].la + g[i].lb - 1, sa = w[i].la, lsh = w[i].lb;
      tj_of[i] = nt;
      tj.j[nt++] = TailJob{w[i].b8, lsh, w[i].a8 + sa, (int)es[i], sa, sa + lsh - 1, rl, g[i].out, {nullptr, nullptr},
                           {nullptr, nullptr}};
      maxspan = std::max<uint64_t>(maxspan, rl - sa);
      continue;
    }
    if (nt && i == m) {
      const uint64_t blocks64 = (maxspan + 16 * 256 - 1) / (16 * 256);
      hipLaunchKernelGGL(polymul_tail_batch_kernel, dim3((unsigned)std::min<uint64_t>(blocks64, 4096), nt), dim3(256), 0,
                         st, tj);
      PLK_HIP(hipGetLastError());
    }
  }
  return PLK_OK;
}

// d_out must hold la+lb-1 bytes; *d_nz (if not NULL) receives the trimmed length (0 means "all zero" ->
// the caller reports length 1).
int plk_poly_mul_launch(const uint8_t* d_a, uint64_t la, const uint8_t* d_b, uint64_t lb, uint8_t* d_out,
                        uint32_t* d_nz, void* d_work, hipStream_t st) {
  if (la == 0 || lb == 0) return PLK_ERR_ARG;
  const uint64_t rl = la + lb - 1;
  const uint64_t mn = la < lb ? la : lb;
  if (mn * 256 >= bb::P) return PLK_ERR_RANGE;
  if (rl >= (1ull << 32)) return PLK_ERR_RANGE;
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
  if (k > bb::TWO_ADICITY) return PLK_ERR_RANGE;
  const uint32_t ninv = bb::hpow(1ull << k, bb::P - 2);   // normal form on purpose
  if (k <= PLK_SMALL_LOG) {   // (never split: product_plan only splits above 2^(SMALL_LOG+1))
    const size_t lds = (size_t)4 * (2 * col_stride(1 << k) + 2 * (1 << k));
    hipLaunchKernelGGL(polymul_small_kernel, dim3(1), dim3(1024), lds, st, d_a, la, d_b, lb, k, tw_fwd(), tw_inv(),
                       d_out, ninv, d_nz);
    PLK_HIP(hipGetLastError());
    return PLK_OK;
  }
  if (!d_work) return PLK_ERR_ARG;
  const PlkPolyMulJob job{d_a, la, d_b, lb, d_out};
  int rc = ntt_group(&job, 1, k, e ? &e : nullptr, d_work, st);
  if (rc) return rc;
  if (d_nz) hipLaunchKernelGGL(trim_kernel, dim3(1), dim3(1024), 0, st, d_out, rl, d_nz);
  PLK_HIP(hipGetLastError());
  return PLK_OK;
}

// Several independent products: direct / one-workgroup ones one by one, the NTT ones grouped
// by transform size and run as batches through the wave engine (one launch per pass for the
// whole group; job i of a group uses 2^(k+3) bytes of d_work at offset i 2^(k+3)).  The
// prover's round-3 products come in such groups (7 at 2^21, then 3 + 2 at 2^22 for n = 2^20).
int plk_poly_mul_batch_launch(const PlkPolyMulJob* jobs, int nj, void* d_work, size_t work_bytes, hipStream_t st) {
  int ks[64];
  uint64_t es[64];
  if (nj > 64) {
    plk_set_error("poly_mul batch of %d products (max 64)", nj);
    return PLK_ERR_RANGE;
  }
  for (int i = 0; i < nj; i++) {
    const PlkPolyMulJob& j = jobs[i];
    ks[i] = -1;
    if (j.la == 0 || j.lb == 0) return PLK_ERR_ARG;
    const uint64_t mn = j.la < j.lb ? j.la : j.lb;
    const int k = product_plan(j.la, j.lb, &es[i]);
    if (j.acc && !(mn > PLK_DIRECT_MAX && k > PLK_SMALL_LOG)) {
      plk_set_error("poly_mul batch: sum-group member %d is not a transform-sized product", i);
      return PLK_ERR_ARG;
    }
    if (mn > PLK_DIRECT_MAX && k > PLK_SMALL_LOG) {
      if (mn * 256 >= bb::P || k > bb::TWO_ADICITY) return PLK_ERR_RANGE;
      ks[i] = k;
      continue;
    }
    const int rc = plk_poly_mul_launch(j.a, j.la, j.b, j.lb, j.out, nullptr, nullptr, st);
    if (rc) return rc;
  }
  bool done[64] = {false};
  for (int i = 0; i < nj; i++) {
    if (ks[i] < 0 || done[i]) continue;
    const int k = ks[i];
    const size_t per = (size_t)8 << k;
    const int cap = (int)(work_bytes / per);
    if (cap < 1) {
      plk_set_error("poly_mul batch: workspace %zu bytes < %zu", work_bytes, per);
      return PLK_ERR_ARG;
    }
    PlkPolyMulJob g[64];
    uint64_t ge[64];
    int m = 0;
    for (int q = i; q < nj && m < cap; q++)
      if (!done[q] && ks[q] == k) {
        g[m] = jobs[q];
        ge[m++] = es[q];
        done[q] = true;
      }
    const int rc = ntt_group(g, m, k, ge, d_work, st);
    if (rc) return rc;
  }
  return PLK_OK;
}

// Standalone forward NTT (DIF, natural -> bit-reversed), in place on Montgomery-form u32,
// or inverse (DIT, bit-reversed -> natural, NOT scaled by N^-1).  Same passes as poly_mul.
// batch independent arrays at d + b 2^k share each pass's launch (up to 12 per launch).
int plk_ntt_launch(uint32_t* d, int k, int batch, int inverse, hipStream_t st) {
  if (k < 1 || k > bb::TWO_ADICITY || batch < 1) return PLK_ERR_RANGE;
  if (plk_wave_ntt_supported(k)) return plk_wave_ntt_launch(d, k, batch, inverse, st);
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
