// Wave-tile NTT passes for transforms of 2^13 .. 2^27 points (poly_mul and plk_ntt_dev).
//
// One WAVE owns one tile of 1024 elements: 2^M rows (the pass's butterfly bits) x
// C = 2^(10-M) columns, 16 elements per lane held in registers.  A pass runs its M radix-2
// stages as radix-16 rounds: a round keeps four consecutive tile bits [lb, lb+4) local to a
// lane (its 16 registers) and the other six bits across the 64 lanes; between rounds the
// wave transposes through its own LDS buffer (no workgroup barrier).  The first round
// loads straight from global memory and the last one stores straight back, so a pass costs
// one read + one write of the array and 1-2 LDS exchanges.
//
// Passes over high bits (lo > 0) need a per-column twiddle w_N^(L * 2^(k-1-s)) at every
// stage s; those factor out of the column transform exactly (checked numerically): a DIF
// pass = plain size-2^M DIF per column, then one multiply of the element at local row r by
// w_{2^(lo+M)}^(L * bitrev_M(r)); a DIT pass = the inverse pre-multiply, then a plain DIT.
//
// Tiles are placed XCD-aware: blocks b and b+8 share an XCD (observed dispatch, speed
// only), so consecutive tile blocks -- which share cache lines in high-bit passes -- are
// handed to blocks with the same b % 8.
#include "plk_device.h"
#include "plk_internal.h"

#include <stdlib.h>

namespace {

constexpr int WT_BITS = 10;                    // tile = 1024 elements
constexpr int WT_BUF = (1 << WT_BITS) + (1 << WT_BITS) / 32;   // padded exchange buffer (words)

__device__ __forceinline__ int wphys(int e) { return e + (e >> 5); }

struct WPass {
  int k;    // log2 N
  int lo;   // lowest bit of the pass
  int M;    // bits of the pass (rows); C = 2^(10 - M) columns
};

struct WTw {
  const uint32_t* small;   // T[2^j + r] = w_{2^(j+1)}^r (Montgomery)
  const uint32_t* lo;      // w_{2^27}^i, i < 4096
  const uint32_t* hi;      // w_{2^27}^(4096 i)
};

__device__ __forceinline__ uint32_t root27(const WTw& t, uint32_t e) {
  return bb::mmul(t.lo[e & 4095u], t.hi[e >> 12]);
}

// global index of tile-local element e = c * 2^M + r
__device__ __forceinline__ uint64_t wt_index(const WPass& p, uint32_t tile, uint32_t e) {
  if (p.lo == 0) return ((uint64_t)tile << WT_BITS) | e;
  const int cb = WT_BITS - p.M;
  const uint32_t r = e & ((1u << p.M) - 1), c = e >> p.M;
  const uint32_t per_h = 1u << (p.lo - cb);
  const uint64_t H = tile / per_h;
  const uint32_t L = ((tile % per_h) << cb) | c;
  return (H << (p.lo + p.M)) | ((uint64_t)r << p.lo) | L;
}

// Tile engine with R local bits per thread (E = 2^R registers, 2^(10-R) threads per tile).
template <int R>
struct Eng {
  static constexpr int E = 1 << R;
  static constexpr int NT = 1 << (WT_BITS - R);

  // element held by (thread, k) in a round with local bits [lb, lb+R): base(thread) + k << lb.
  // cols_first (only when [lb, lb+R) are all row bits): the low thread bits index the
  // columns, so in high-bit passes consecutive threads touch consecutive addresses.
  __device__ static __forceinline__ uint32_t base(uint32_t tid, int lb, int M, bool cols_first) {
    if (!cols_first) return (tid & ((1u << lb) - 1)) | ((tid >> lb) << (lb + R));
    const int cb = WT_BITS - M;
    const uint32_t c = tid & ((1u << cb) - 1), rr = tid >> cb;
    return (c << M) | (rr & ((1u << lb) - 1)) | ((rr >> lb) << (lb + R));
  }

  struct Round {
    int s_lo, s_hi, lb;
  };
  __device__ static __forceinline__ int rounds(int M) { return (M + R - 1) / R; }
  // DIF: chunks of <= R stage bits from the top; DIT: from the bottom.
  __device__ static __forceinline__ Round round_of(int M, int q, bool inv) {
    Round r;
    if (!inv) {
      r.s_hi = M - 1 - R * q;
      r.s_lo = r.s_hi - (R - 1) < 0 ? 0 : r.s_hi - (R - 1);
    } else {
      r.s_lo = R * q;
      r.s_hi = r.s_lo + (R - 1) > M - 1 ? M - 1 : r.s_lo + (R - 1);
    }
    r.lb = r.s_lo < WT_BITS - R ? r.s_lo : WT_BITS - R;
    return r;
  }
  __device__ static __forceinline__ bool cols_first(const WPass& p, const Round& r) {
    return p.lo != 0 && r.lb + R <= p.M;
  }

  // one radix-2 stage on k-bit Q (row bit s = lb + Q)
  template <int Q, bool INV>
  __device__ static __forceinline__ void stage(uint32_t (&v)[E], uint32_t b, int lb, int s, const uint32_t* Tsm) {
    const uint32_t hs = 1u << s;
    const uint32_t b0 = b & ((1u << lb) - 1) & (hs - 1);
#pragma unroll
    for (int k = 0; k < E; k++) {
      if (k & (1 << Q)) continue;
      const uint32_t rr = b0 + ((uint32_t)(k & ((1 << Q) - 1)) << lb);   // row mod 2^s
      const uint32_t w = Tsm[hs + rr];
      const uint32_t u = v[k], x = v[k | (1 << Q)];
      if (!INV) {
        v[k] = bb::madd(u, x);
        v[k | (1 << Q)] = bb::mmul(bb::msub(u, x), w);
      } else {
        const uint32_t xw = bb::mmul(x, w);
        v[k] = bb::madd(u, xw);
        v[k | (1 << Q)] = bb::msub(u, xw);
      }
    }
  }

  template <bool INV>
  __device__ static __forceinline__ void stage_q(uint32_t (&v)[E], uint32_t b, int lb, int s, const uint32_t* Tsm) {
    const int q = s - lb;
    if (R > 3 && q == 3) stage<(R > 3 ? 3 : 0), INV>(v, b, lb, s, Tsm);
    else if (R > 2 && q == 2) stage<(R > 2 ? 2 : 0), INV>(v, b, lb, s, Tsm);
    else if (R > 1 && q == 1) stage<(R > 1 ? 1 : 0), INV>(v, b, lb, s, Tsm);
    else stage<0, INV>(v, b, lb, s, Tsm);
  }

  template <bool INV>
  __device__ static __forceinline__ void round_compute(uint32_t (&v)[E], const Round& r, uint32_t b,
                                                       const uint32_t* Tsm) {
    if (!INV) {
      for (int s = r.s_hi; s >= r.s_lo; s--) stage_q<false>(v, b, r.lb, s, Tsm);
    } else {
      for (int s = r.s_lo; s <= r.s_hi; s++) stage_q<true>(v, b, r.lb, s, Tsm);
    }
  }

  // registers (mapping from) -> LDS -> registers (mapping to).  Double-buffered, so one
  // barrier per exchange suffices: the buffer written next was last read before the
  // previous barrier.
  __device__ static __forceinline__ void exchange(uint32_t (&v)[E], uint32_t* buf, uint32_t bf, int lbf,
                                                  uint32_t bt, int lbt) {
#pragma unroll
    for (int k = 0; k < E; k++) buf[wphys((int)(bf + ((uint32_t)k << lbf)))] = v[k];
    if (NT > 64) __syncthreads();
    else { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); __builtin_amdgcn_wave_barrier(); }
#pragma unroll
    for (int k = 0; k < E; k++) v[k] = buf[wphys((int)(bt + ((uint32_t)k << lbt)))];
  }

  // All rounds of one pass on registers holding the round-0 mapping; bufs = 2 x WT_BUF
  // words, *xc counts exchanges (selects the buffer).  Leaves the final mapping in b_io/lb_io.
  template <bool INV>
  __device__ static __forceinline__ void pass(uint32_t (&v)[E], const WPass& p, uint32_t tid, uint32_t* bufs,
                                              int& xc, const uint32_t* Tsm, uint32_t& b_io, int& lb_io) {
    const int nr = rounds(p.M);
    Round r = round_of(p.M, 0, INV);
    uint32_t b = base(tid, r.lb, p.M, cols_first(p, r));
    round_compute<INV>(v, r, b, Tsm);
    for (int q = 1; q < nr; q++) {
      const Round rn = round_of(p.M, q, INV);
      const uint32_t bn = base(tid, rn.lb, p.M, (q == nr - 1) && cols_first(p, rn));
      exchange(v, bufs + (xc++ & 1) * WT_BUF, b, r.lb, bn, rn.lb);
      r = rn;
      b = bn;
      round_compute<INV>(v, r, b, Tsm);
    }
    b_io = b;
    lb_io = r.lb;
  }
};

// tile of this block, XCD-aware: consecutive tiles go to blocks with equal b % 8
__device__ __forceinline__ uint32_t block_tile() {
  const uint32_t nb = gridDim.x, b = blockIdx.x;
  return (nb % 8 == 0) ? (b % 8) * (nb / 8) + b / 8 : b;
}

// column factor exponent (in w_{2^27} units) for element e of a high-bit pass
__device__ __forceinline__ uint32_t col_exp(const WPass& p, uint32_t tile, uint32_t e) {
  const int cb = WT_BITS - p.M;
  const uint32_t r = e & ((1u << p.M) - 1), c = e >> p.M;
  const uint32_t per_h = 1u << (p.lo - cb);
  const uint32_t L = ((tile % per_h) << cb) | c;
  const uint32_t f = __brev(r) >> (32 - p.M);
  return (L * f) << (27 - p.lo - p.M);   // w_{2^(lo+M)}^(L f); L f < 2^(lo+M)
}

__device__ __forceinline__ void load_small_tw(uint32_t* Tsm, const uint32_t* small, int M) {
  for (int i = threadIdx.x; i < (1 << M); i += blockDim.x) Tsm[i] = small[i];
}

}  // namespace

// Forward (DIF) pass over 1 or 2 arrays (blockIdx.y), u32 in place, or the first pass
// reading bytes (zero padded, reduced mod 17, to Montgomery).
template <int R, bool FROM_U8>
__global__ __launch_bounds__(Eng<R>::NT) void wt_fwd_kernel(WPass p, uint32_t* d0, uint32_t* d1, const uint8_t* a8,
                                                            const uint8_t* b8, uint64_t la, uint64_t lb8, WTw tw) {
  using G = Eng<R>;
  __shared__ uint32_t Tsm[1 << WT_BITS];
  __shared__ uint32_t bufs[2 * WT_BUF];
  const uint32_t tid = threadIdx.x;
  const uint32_t tile = block_tile();
  uint32_t* d = blockIdx.y == 0 ? d0 : d1;
  const uint8_t* s8 = blockIdx.y == 0 ? a8 : b8;
  const uint64_t ls = blockIdx.y == 0 ? la : lb8;

  const auto r0 = G::round_of(p.M, 0, false);
  const uint32_t b0 = G::base(tid, r0.lb, p.M, G::cols_first(p, r0));
  uint32_t v[G::E];
#pragma unroll
  for (int k = 0; k < G::E; k++) {
    const uint64_t idx = wt_index(p, tile, b0 + ((uint32_t)k << r0.lb));
    if (FROM_U8) v[k] = idx < ls ? bb::mmul((uint32_t)(s8[idx] % 17u), bb::R2) : 0u;
    else v[k] = d[idx];
  }
  load_small_tw(Tsm, tw.small, p.M);
  __syncthreads();
  uint32_t b;
  int lbf, xc = 0;
  G::template pass<false>(v, p, tid, bufs, xc, Tsm, b, lbf);
#pragma unroll
  for (int k = 0; k < G::E; k++) {
    const uint32_t e = b + ((uint32_t)k << lbf);
    uint32_t x = v[k];
    if (p.lo != 0) x = bb::mmul(x, root27(tw, col_exp(p, tile, e)));
    d[wt_index(p, tile, e)] = x;
  }
}

// Inverse (DIT) pass, u32 in place; the final pass (TO_U8) scales by N^-1 (normal form,
// which also leaves Montgomery form), reduces mod 17, writes bytes for idx < out_len and
// the max non-zero index + 1 to *nz.
template <int R, bool TO_U8>
__global__ __launch_bounds__(Eng<R>::NT) void wt_inv_kernel(WPass p, uint32_t* d, WTw tw, uint8_t* out8,
                                                            uint64_t out_len, uint32_t ninv, uint32_t* nz) {
  using G = Eng<R>;
  __shared__ uint32_t Tsm[1 << WT_BITS];
  __shared__ uint32_t bufs[2 * WT_BUF];
  const uint32_t tid = threadIdx.x;
  const uint32_t tile = block_tile();

  const auto r0 = G::round_of(p.M, 0, true);
  const uint32_t b0 = G::base(tid, r0.lb, p.M, G::cols_first(p, r0));
  uint32_t v[G::E];
#pragma unroll
  for (int k = 0; k < G::E; k++) {
    const uint32_t e = b0 + ((uint32_t)k << r0.lb);
    uint32_t x = d[wt_index(p, tile, e)];
    if (p.lo != 0) x = bb::mmul(x, root27(tw, col_exp(p, tile, e)));   // tw = inverse roots
    v[k] = x;
  }
  load_small_tw(Tsm, tw.small, p.M);
  __syncthreads();
  uint32_t b;
  int lbf, xc = 0;
  G::template pass<true>(v, p, tid, bufs, xc, Tsm, b, lbf);
  uint32_t last = 0;
#pragma unroll
  for (int k = 0; k < G::E; k++) {
    const uint64_t idx = wt_index(p, tile, b + ((uint32_t)k << lbf));
    if (!TO_U8) {
      d[idx] = v[k];
    } else if (idx < out_len) {
      const uint8_t byte = (uint8_t)(bb::mmul(v[k], ninv) % 17u);
      out8[idx] = byte;
      if (byte && (uint32_t)idx + 1 > last) last = (uint32_t)idx + 1;
    }
  }
  if (TO_U8) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) last = max(last, (uint32_t)__shfl_xor(last, off, PLK_WAVE));
    if ((tid & 63u) == 0 && last) atomicMax(nz, last);
  }
}

// Center of poly_mul: last forward pass (lo = 0) of a and b, pointwise product, first
// inverse pass, all in registers of one block; result written over a.
template <int R>
__global__ __launch_bounds__(Eng<R>::NT) void wt_center_kernel(WPass p, uint32_t* d0, const uint32_t* d1, WTw twf,
                                                               WTw twi) {
  using G = Eng<R>;
  __shared__ uint32_t Tf[1 << WT_BITS];
  __shared__ uint32_t Ti[1 << WT_BITS];
  __shared__ uint32_t bufs[2 * WT_BUF];
  const uint32_t tid = threadIdx.x;
  const uint32_t tile = block_tile();
  const auto r0 = G::round_of(p.M, 0, false);
  const uint32_t b0 = G::base(tid, r0.lb, p.M, false);
  uint32_t va[G::E], vb[G::E];
#pragma unroll
  for (int k = 0; k < G::E; k++) {
    const uint64_t idx = wt_index(p, tile, b0 + ((uint32_t)k << r0.lb));
    va[k] = d0[idx];
    vb[k] = d1[idx];
  }
  load_small_tw(Tf, twf.small, p.M);
  load_small_tw(Ti, twi.small, p.M);
  __syncthreads();
  uint32_t ba, bb_;
  int la_, lb_, xc = 0;
  G::template pass<false>(va, p, tid, bufs, xc, Tf, ba, la_);
  G::template pass<false>(vb, p, tid, bufs, xc, Tf, bb_, lb_);
#pragma unroll
  for (int k = 0; k < G::E; k++) va[k] = bb::mmul(va[k], vb[k]);
  const auto i0 = G::round_of(p.M, 0, true);
  const uint32_t bi = G::base(tid, i0.lb, p.M, false);
  if (ba != bi || la_ != i0.lb) G::exchange(va, bufs + (xc++ & 1) * WT_BUF, ba, la_, bi, i0.lb);
  uint32_t b;
  int lbf;
  G::template pass<true>(va, p, tid, bufs, xc, Ti, b, lbf);
#pragma unroll
  for (int k = 0; k < G::E; k++) d0[wt_index(p, tile, b + ((uint32_t)k << lbf))] = va[k];
}

// ------------------------------------------------------------------------------ host side
namespace {

// passes of a 2^k transform, high bits first: the remainder pass (k mod 10 bits, many
// columns -> long contiguous rows) on top, then 10-bit passes down to the lo = 0 pass
int wave_plan(int k, int* Ms) {
  int n = 0, left = k;
  while (left > 0) {
    const int m = left > 10 ? (left - 1) % 10 + 1 : left;
    Ms[n++] = m;
    left -= m;
  }
  return n;
}

WTw to_wtw(const PlkTwTables& t, bool inv) {
  return inv ? WTw{t.small_i, t.lo_i, t.hi_i} : WTw{t.small_f, t.lo_f, t.hi_f};
}

}  // namespace

static int wt_radix_bits() {
  static int r = -1;
  if (r < 0) {
    const char* e = getenv("PLK_NTT_RADIX_BITS");
    r = e ? atoi(e) : 2;
    if (r < 1 || r > 4) r = 2;
  }
  return r;
}

bool plk_wave_ntt_supported(int k) { return k >= 13 && k <= bb::TWO_ADICITY; }

template <int R>
static int wave_poly_mul_r(const uint8_t* d_a, uint64_t la, const uint8_t* d_b, uint64_t lb, int k, uint8_t* d_out,
                           uint32_t* d_nz, uint32_t* A, uint32_t* B, uint32_t ninv, hipStream_t st) {
  const PlkTwTables t = plk_ntt_tables();
  const WTw twf = to_wtw(t, false), twi = to_wtw(t, true);
  int Ms[4];
  const int np = wave_plan(k, Ms);
  int lo[4];
  for (int i = 0, top = k; i < np; i++) { lo[i] = top - Ms[i]; top = lo[i]; }
  const uint32_t tiles = (uint32_t)((1ull << k) >> WT_BITS);
  const dim3 blk(Eng<R>::NT);
  for (int i = 0; i < np - 1; i++) {
    const WPass p{k, lo[i], Ms[i]};
    if (i == 0)
      hipLaunchKernelGGL((wt_fwd_kernel<R, true>), dim3(tiles, 2), blk, 0, st, p, A, B, d_a, d_b, la, lb, twf);
    else
      hipLaunchKernelGGL((wt_fwd_kernel<R, false>), dim3(tiles, 2), blk, 0, st, p, A, B, nullptr, nullptr,
                         (uint64_t)0, (uint64_t)0, twf);
    PLK_HIP(hipGetLastError());
  }
  hipLaunchKernelGGL((wt_center_kernel<R>), dim3(tiles), blk, 0, st, WPass{k, 0, Ms[np - 1]}, A, B, twf, twi);
  PLK_HIP(hipGetLastError());
  const uint64_t rl = la + lb - 1;
  for (int i = np - 2; i >= 0; i--) {
    const WPass p{k, lo[i], Ms[i]};
    if (i == 0)
      hipLaunchKernelGGL((wt_inv_kernel<R, true>), dim3(tiles), blk, 0, st, p, A, twi, d_out, rl, ninv, d_nz);
    else
      hipLaunchKernelGGL((wt_inv_kernel<R, false>), dim3(tiles), blk, 0, st, p, A, twi, nullptr, (uint64_t)0, 0u,
                         nullptr);
    PLK_HIP(hipGetLastError());
  }
  return PLK_OK;
}

int plk_wave_poly_mul_launch(const uint8_t* d_a, uint64_t la, const uint8_t* d_b, uint64_t lb, int k,
                             uint8_t* d_out, uint32_t* d_nz, uint32_t* A, uint32_t* B, uint32_t ninv, hipStream_t st) {
  switch (wt_radix_bits()) {
    case 1: return wave_poly_mul_r<1>(d_a, la, d_b, lb, k, d_out, d_nz, A, B, ninv, st);
    case 3: return wave_poly_mul_r<3>(d_a, la, d_b, lb, k, d_out, d_nz, A, B, ninv, st);
    case 4: return wave_poly_mul_r<4>(d_a, la, d_b, lb, k, d_out, d_nz, A, B, ninv, st);
    default: return wave_poly_mul_r<2>(d_a, la, d_b, lb, k, d_out, d_nz, A, B, ninv, st);
  }
}

template <int R>
static int wave_ntt_r(uint32_t* d, int k, int inverse, hipStream_t st) {
  const PlkTwTables t = plk_ntt_tables();
  int Ms[4];
  const int np = wave_plan(k, Ms);
  int lo[4];
  for (int i = 0, top = k; i < np; i++) { lo[i] = top - Ms[i]; top = lo[i]; }
  const uint32_t tiles = (uint32_t)((1ull << k) >> WT_BITS);
  const dim3 blk(Eng<R>::NT);
  for (int s = 0; s < np; s++) {
    const int i = inverse ? np - 1 - s : s;
    const WPass p{k, lo[i], Ms[i]};
    if (inverse)
      hipLaunchKernelGGL((wt_inv_kernel<R, false>), dim3(tiles), blk, 0, st, p, d, to_wtw(t, true), nullptr,
                         (uint64_t)0, 0u, nullptr);
    else
      hipLaunchKernelGGL((wt_fwd_kernel<R, false>), dim3(tiles, 1), blk, 0, st, p, d, d, nullptr, nullptr,
                         (uint64_t)0, (uint64_t)0, to_wtw(t, false));
    PLK_HIP(hipGetLastError());
  }
  return PLK_OK;
}

int plk_wave_ntt_launch(uint32_t* d, int k, int inverse, hipStream_t st) {
  switch (wt_radix_bits()) {
    case 1: return wave_ntt_r<1>(d, k, inverse, st);
    case 3: return wave_ntt_r<3>(d, k, inverse, st);
    case 4: return wave_ntt_r<4>(d, k, inverse, st);
    default: return wave_ntt_r<2>(d, k, inverse, st);
  }
}
