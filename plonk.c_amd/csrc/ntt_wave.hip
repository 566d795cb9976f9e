// Tile-engine NTT passes for transforms of 2^13 .. 2^27 points (poly_mul and plk_ntt_dev).
//
// One block owns one tile of 4096 elements: 2^M rows (the pass's butterfly bits) x
// C = 2^(12-M) columns.  Each thread holds E = 2^R elements in registers (R = 2 by default,
// PLK_NTT_RADIX_BITS): a round keeps R consecutive tile bits [lb, lb+R) local to a thread
// and the other 12-R bits across the block's threads, runs its (<= R) radix-2 stages in
// registers, and the block transposes through a double-buffered, padded LDS buffer between
// rounds (one barrier each).  The first round loads straight from global memory and the
// last one stores straight back: a pass costs one read + one write of the array.
// M is a template parameter, so every round, stage and register index is a compile-time
// constant (no private-memory spills of the register tile).
//
// Plan: the lo = 0 pass takes the low 12 bits (contiguous tiles); the bits above are split
// into passes of <= 8 bits, so every high-bit pass has >= 16 contiguous columns (64 B rows).
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

constexpr int WT_BITS = 12;                    // tile = 4096 elements
constexpr int WT_BUF = (1 << WT_BITS) + (1 << WT_BITS) / 32;   // padded exchange buffer (words)
constexpr int WT_MAX_HI = 8;                   // widest high-bit pass

__device__ __forceinline__ int wphys(int e) { return e + (e >> 5); }

struct WPass {
  int k;    // log2 N
  int lo;   // lowest bit of the pass
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
template <int M>
__device__ __forceinline__ uint64_t wt_index(const WPass& p, uint32_t tile, uint32_t e) {
  if (M == WT_BITS) return ((uint64_t)tile << WT_BITS) | e;
  constexpr int cb = WT_BITS - M;
  const uint32_t r = e & ((1u << M) - 1), c = e >> M;
  const uint32_t per_h = 1u << (p.lo - cb);
  const uint64_t H = tile / per_h;
  const uint32_t L = ((tile % per_h) << cb) | c;
  return (H << (p.lo + M)) | ((uint64_t)r << p.lo) | L;
}

// Tile engine with R local bits per thread (E = 2^R registers, 2^(12-R) threads per tile)
// for a pass of M row bits.  HIGH = the pass is over high index bits (lo > 0): exactly the
// passes with M < 12.
template <int R, int M>
struct Eng {
  static constexpr int E = 1 << R;
  static constexpr int NT = 1 << (WT_BITS - R);
  static constexpr bool HIGH = M < WT_BITS;
  static constexpr int NR = (M + R - 1) / R;   // rounds

  // DIF rounds take chunks of <= R stage bits from the top, DIT rounds from the bottom.
  static constexpr int s_hi(int q, bool inv) {
    return inv ? (R * q + R - 1 > M - 1 ? M - 1 : R * q + R - 1) : M - 1 - R * q;
  }
  static constexpr int s_lo(int q, bool inv) {
    return inv ? R * q : (M - 1 - R * q - (R - 1) < 0 ? 0 : M - 1 - R * q - (R - 1));
  }
  static constexpr int lbq(int q, bool inv) { return s_lo(q, inv) < WT_BITS - R ? s_lo(q, inv) : WT_BITS - R; }
  // first/last round of a high-bit pass: the low thread bits index the columns, so
  // consecutive threads touch consecutive global addresses.
  static constexpr bool colsq(int q, bool inv) { return HIGH && (q == 0 || q == NR - 1) && lbq(q, inv) + R <= M; }

  // element held by (thread, k) in a round with local bits [lb, lb+R): base(thread) + k << lb
  __device__ static __forceinline__ uint32_t base(uint32_t tid, int lb, bool cols_first) {
    if (!cols_first) return (tid & ((1u << lb) - 1)) | ((tid >> lb) << (lb + R));
    constexpr int cb = WT_BITS - M;
    const uint32_t c = tid & ((1u << cb) - 1), rr = tid >> cb;
    return (c << M) | (rr & ((1u << lb) - 1)) | ((rr >> lb) << (lb + R));
  }
  template <int Q>
  __device__ static __forceinline__ uint32_t base_q(uint32_t tid, bool inv) {
    return base(tid, lbq(Q, inv), colsq(Q, inv));
  }

  // the radix-2 stages of round Q, in registers
  template <int Q, bool INV>
  __device__ static __forceinline__ void round(uint32_t (&v)[E], uint32_t b, const uint32_t* Tsm) {
    constexpr int LB = lbq(Q, INV), SL = s_lo(Q, INV), SH = s_hi(Q, INV);
    const uint32_t blow = b & ((1u << LB) - 1);
#pragma unroll
    for (int i = 0; i <= SH - SL; i++) {
      const int s = INV ? SL + i : SH - i;
      const int q = s - LB;
#pragma unroll
      for (int k = 0; k < E; k++) {
        if (k & (1 << q)) continue;
        const uint32_t rr = blow + ((uint32_t)(k & ((1 << q) - 1)) << LB);   // row mod 2^s
        const uint32_t w = Tsm[(1u << s) + rr];
        const uint32_t u = v[k], x = v[k | (1 << q)];
        if (!INV) {
          v[k] = bb::madd(u, x);
          v[k | (1 << q)] = bb::mmul(bb::msub(u, x), w);
        } else {
          const uint32_t xw = bb::mmul(x, w);
          v[k] = bb::madd(u, xw);
          v[k | (1 << q)] = bb::msub(u, xw);
        }
      }
    }
  }

  // registers (mapping from) -> LDS -> registers (mapping to).  Double-buffered, so one
  // barrier per exchange suffices: the buffer written next was last read before the
  // previous barrier.
  __device__ static __forceinline__ void exchange(uint32_t (&v)[E], uint32_t* buf, uint32_t bf, int lbf, uint32_t bt,
                                                  int lbt) {
#pragma unroll
    for (int k = 0; k < E; k++) buf[wphys((int)(bf + ((uint32_t)k << lbf)))] = v[k];
    __syncthreads();
#pragma unroll
    for (int k = 0; k < E; k++) v[k] = buf[wphys((int)(bt + ((uint32_t)k << lbt)))];
  }

  // rounds Q .. NR-1 of a pass; registers hold the mapping of round Q on entry and of the
  // last round on exit.  xc selects the exchange buffer (it counts exchanges).
  template <bool INV, int Q = 0>
  __device__ static __forceinline__ void pass(uint32_t (&v)[E], uint32_t tid, uint32_t* bufs, int xc,
                                              const uint32_t* Tsm) {
    round<Q, INV>(v, base_q<Q>(tid, INV), Tsm);
    if constexpr (Q + 1 < NR) {
      exchange(v, bufs + ((xc + Q) & 1) * WT_BUF, base_q<Q>(tid, INV), lbq(Q, INV), base_q<Q + 1>(tid, INV),
               lbq(Q + 1, INV));
      pass<INV, Q + 1>(v, tid, bufs, xc, Tsm);
    }
  }
  static constexpr int XCH = NR - 1;   // exchanges per pass
};

// tile of this block, XCD-aware: consecutive tiles go to blocks with equal b % 8
__device__ __forceinline__ uint32_t block_tile() {
  const uint32_t nb = gridDim.x, b = blockIdx.x;
  return (nb % 8 == 0) ? (b % 8) * (nb / 8) + b / 8 : b;
}

// column factor exponent (in w_{2^27} units) for element e of a high-bit pass
template <int M>
__device__ __forceinline__ uint32_t col_exp(const WPass& p, uint32_t tile, uint32_t e) {
  constexpr int cb = WT_BITS - M;
  const uint32_t r = e & ((1u << M) - 1), c = e >> M;
  const uint32_t per_h = 1u << (p.lo - cb);
  const uint32_t L = ((tile % per_h) << cb) | c;
  const uint32_t f = __brev(r) >> (32 - M);
  return (L * f) << (27 - p.lo - M);   // w_{2^(lo+M)}^(L f); L f < 2^(lo+M)
}

template <int M, int NT>
__device__ __forceinline__ void load_small_tw(uint32_t* Tsm, const uint32_t* small) {
#pragma unroll
  for (int i = 0; i < ((1 << M) + NT - 1) / NT; i++) {
    const int j = i * NT + (int)threadIdx.x;
    if (j < (1 << M)) Tsm[j] = small[j];
  }
}

}  // namespace

// Forward (DIF) pass over 1 or 2 arrays (blockIdx.y), u32 in place, or the first pass
// reading bytes (zero padded, reduced mod 17, to Montgomery).
template <int R, int M, bool FROM_U8>
__global__ __launch_bounds__((Eng<R, M>::NT)) void wt_fwd_kernel(WPass p, uint32_t* d0, uint32_t* d1, const uint8_t* a8,
                                                               const uint8_t* b8, uint64_t la, uint64_t lb8, WTw tw) {
  using G = Eng<R, M>;
  __shared__ uint32_t Tsm[1 << M];
  __shared__ uint32_t bufs[G::XCH == 0 ? 1 : (G::XCH > 1 ? 2 : 1) * WT_BUF];
  const uint32_t tid = threadIdx.x;
  const uint32_t tile = block_tile();
  uint32_t* d = blockIdx.y == 0 ? d0 : d1;
  const uint8_t* s8 = blockIdx.y == 0 ? a8 : b8;
  const uint64_t ls = blockIdx.y == 0 ? la : lb8;

  const uint32_t b0 = G::template base_q<0>(tid, false);
  constexpr int L0 = G::lbq(0, false);
  uint32_t v[G::E];
#pragma unroll
  for (int k = 0; k < G::E; k++) {
    const uint64_t idx = wt_index<M>(p, tile, b0 + ((uint32_t)k << L0));
    if (FROM_U8) v[k] = idx < ls ? bb::mmul((uint32_t)(s8[idx] % 17u), bb::R2) : 0u;
    else v[k] = d[idx];
  }
  load_small_tw<M, G::NT>(Tsm, tw.small);
  __syncthreads();
  G::template pass<false>(v, tid, bufs, 0, Tsm);
  constexpr int LF = G::lbq(G::NR - 1, false);
  const uint32_t bf = G::template base_q<G::NR - 1>(tid, false);
#pragma unroll
  for (int k = 0; k < G::E; k++) {
    const uint32_t e = bf + ((uint32_t)k << LF);
    uint32_t x = v[k];
    if (G::HIGH) x = bb::mmul(x, root27(tw, col_exp<M>(p, tile, e)));
    d[wt_index<M>(p, tile, e)] = x;
  }
}

// Inverse (DIT) pass, u32 in place; the final pass (TO_U8) scales by N^-1 (normal form,
// which also leaves Montgomery form), reduces mod 17 and writes bytes for idx < out_len
// (the trimmed length comes from trim_kernel).
template <int R, int M, bool TO_U8>
__global__ __launch_bounds__((Eng<R, M>::NT)) void wt_inv_kernel(WPass p, uint32_t* d, WTw tw, uint8_t* out8,
                                                               uint64_t out_len, uint32_t ninv) {
  using G = Eng<R, M>;
  __shared__ uint32_t Tsm[1 << M];
  __shared__ uint32_t bufs[G::XCH == 0 ? 1 : (G::XCH > 1 ? 2 : 1) * WT_BUF];
  const uint32_t tid = threadIdx.x;
  const uint32_t tile = block_tile();

  const uint32_t b0 = G::template base_q<0>(tid, true);
  constexpr int L0 = G::lbq(0, true);
  uint32_t v[G::E];
#pragma unroll
  for (int k = 0; k < G::E; k++) {
    const uint32_t e = b0 + ((uint32_t)k << L0);
    uint32_t x = d[wt_index<M>(p, tile, e)];
    if (G::HIGH) x = bb::mmul(x, root27(tw, col_exp<M>(p, tile, e)));   // tw = inverse roots
    v[k] = x;
  }
  load_small_tw<M, G::NT>(Tsm, tw.small);
  __syncthreads();
  G::template pass<true>(v, tid, bufs, 0, Tsm);
  constexpr int LF = G::lbq(G::NR - 1, true);
  const uint32_t bf = G::template base_q<G::NR - 1>(tid, true);
#pragma unroll
  for (int k = 0; k < G::E; k++) {
    const uint64_t idx = wt_index<M>(p, tile, bf + ((uint32_t)k << LF));
    if (!TO_U8) d[idx] = v[k];
    else if (idx < out_len) out8[idx] = (uint8_t)(bb::mmul(v[k], ninv) % 17u);
  }
}

// Center of poly_mul: last forward pass (lo = 0) of a and b, pointwise product, first
// inverse pass, all in registers of one block; result written over a.  The last DIF round
// and the first DIT round both have local bits [0, R), so no exchange sits in between.
template <int R>
__global__ __launch_bounds__((Eng<R, WT_BITS>::NT)) void wt_center_kernel(WPass p, uint32_t* d0, const uint32_t* d1,
                                                                         WTw twf, WTw twi) {
  using G = Eng<R, WT_BITS>;
  static_assert(G::lbq(G::NR - 1, false) == 0 && G::lbq(0, true) == 0, "center mapping");
  __shared__ uint32_t Tf[1 << WT_BITS];
  __shared__ uint32_t Ti[1 << WT_BITS];
  __shared__ uint32_t bufs[2 * WT_BUF];
  const uint32_t tid = threadIdx.x;
  const uint32_t tile = block_tile();
  const uint32_t b0 = G::template base_q<0>(tid, false);
  constexpr int L0 = G::lbq(0, false);
  uint32_t va[G::E], vb[G::E];
#pragma unroll
  for (int k = 0; k < G::E; k++) {
    const uint64_t idx = wt_index<WT_BITS>(p, tile, b0 + ((uint32_t)k << L0));
    va[k] = d0[idx];
    vb[k] = d1[idx];
  }
  load_small_tw<WT_BITS, G::NT>(Tf, twf.small);
  load_small_tw<WT_BITS, G::NT>(Ti, twi.small);
  __syncthreads();
  G::template pass<false>(va, tid, bufs, 0, Tf);
  G::template pass<false>(vb, tid, bufs, G::XCH, Tf);
#pragma unroll
  for (int k = 0; k < G::E; k++) va[k] = bb::mmul(va[k], vb[k]);
  G::template pass<true>(va, tid, bufs, 2 * G::XCH, Ti);
  constexpr int LF = G::lbq(G::NR - 1, true);
  const uint32_t bf = G::template base_q<G::NR - 1>(tid, true);
#pragma unroll
  for (int k = 0; k < G::E; k++) d0[wt_index<WT_BITS>(p, tile, bf + ((uint32_t)k << LF))] = va[k];
}

// ------------------------------------------------------------------------------ host side
namespace {

// passes of a 2^k transform, high bits first: the bits above the 12-bit lo = 0 pass in
// balanced chunks of <= 8 (>= 16 columns per tile row)
int wave_plan(int k, int* Ms) {
  const int hi = k - WT_BITS;
  const int nh = (hi + WT_MAX_HI - 1) / WT_MAX_HI;
  int n = 0;
  for (int i = 0; i < nh; i++) Ms[n++] = hi / nh + (i < hi % nh ? 1 : 0);
  Ms[n++] = WT_BITS;
  return n;
}

WTw to_wtw(const PlkTwTables& t, bool inv) {
  return inv ? WTw{t.small_i, t.lo_i, t.hi_i} : WTw{t.small_f, t.lo_f, t.hi_f};
}

// host launchers, one per (R, M); Ms are 1..8 or 12
template <int R, int M, bool U8>
void launch_fwd(WPass p, uint32_t* d0, uint32_t* d1, const uint8_t* a8, const uint8_t* b8, uint64_t la, uint64_t lb,
                WTw tw, int arrays, hipStream_t st) {
  const uint32_t tiles = (uint32_t)((1ull << p.k) >> WT_BITS);
  hipLaunchKernelGGL((wt_fwd_kernel<R, M, U8>), dim3(tiles, arrays), dim3(Eng<R, M>::NT), 0, st, p, d0, d1, a8, b8,
                     la, lb, tw);
}
template <int R, int M, bool U8>
void launch_inv(WPass p, uint32_t* d, WTw tw, uint8_t* out8, uint64_t out_len, uint32_t ninv, hipStream_t st) {
  const uint32_t tiles = (uint32_t)((1ull << p.k) >> WT_BITS);
  hipLaunchKernelGGL((wt_inv_kernel<R, M, U8>), dim3(tiles), dim3(Eng<R, M>::NT), 0, st, p, d, tw, out8, out_len,
                     ninv);
}

template <int R, bool U8>
int fwd_m(int M, WPass p, uint32_t* d0, uint32_t* d1, const uint8_t* a8, const uint8_t* b8, uint64_t la, uint64_t lb,
          WTw tw, int arrays, hipStream_t st) {
  switch (M) {
#define PLK_FWD_CASE(m) \
  case m: launch_fwd<R, m, U8>(p, d0, d1, a8, b8, la, lb, tw, arrays, st); break;
    PLK_FWD_CASE(1) PLK_FWD_CASE(2) PLK_FWD_CASE(3) PLK_FWD_CASE(4)
    PLK_FWD_CASE(5) PLK_FWD_CASE(6) PLK_FWD_CASE(7) PLK_FWD_CASE(8)
#undef PLK_FWD_CASE
    case WT_BITS:
      if (U8) { plk_set_error("wave plan: first pass cannot be the 12-bit pass"); return PLK_ERR_ARG; }
      launch_fwd<R, WT_BITS, false>(p, d0, d1, a8, b8, la, lb, tw, arrays, st);
      break;
    default: plk_set_error("wave plan: unsupported pass width %d", M); return PLK_ERR_ARG;
  }
  PLK_HIP(hipGetLastError());
  return PLK_OK;
}

template <int R, bool U8>
int inv_m(int M, WPass p, uint32_t* d, WTw tw, uint8_t* out8, uint64_t out_len, uint32_t ninv, hipStream_t st) {
  switch (M) {
#define PLK_INV_CASE(m) \
  case m: launch_inv<R, m, U8>(p, d, tw, out8, out_len, ninv, st); break;
    PLK_INV_CASE(1) PLK_INV_CASE(2) PLK_INV_CASE(3) PLK_INV_CASE(4)
    PLK_INV_CASE(5) PLK_INV_CASE(6) PLK_INV_CASE(7) PLK_INV_CASE(8)
#undef PLK_INV_CASE
    case WT_BITS:
      if (U8) { plk_set_error("wave plan: last pass cannot be the 12-bit pass"); return PLK_ERR_ARG; }
      launch_inv<R, WT_BITS, false>(p, d, tw, out8, out_len, ninv, st);
      break;
    default: plk_set_error("wave plan: unsupported pass width %d", M); return PLK_ERR_ARG;
  }
  PLK_HIP(hipGetLastError());
  return PLK_OK;
}

}  // namespace

static int wt_radix_bits() {
  static int r = -1;
  if (r < 0) {
    const char* e = getenv("PLK_NTT_RADIX_BITS");
    r = e ? atoi(e) : 2;
    if (r < 2 || r > 4) r = 2;   // 2^(12-R) threads per block must be <= 1024
  }
  return r;
}

bool plk_wave_ntt_supported(int k) { return k > WT_BITS && k <= bb::TWO_ADICITY; }

template <int R>
static int wave_poly_mul_r(const uint8_t* d_a, uint64_t la, const uint8_t* d_b, uint64_t lb, int k, uint8_t* d_out,
                           uint32_t* A, uint32_t* B, uint32_t ninv, hipStream_t st) {
  const PlkTwTables t = plk_ntt_tables();
  const WTw twf = to_wtw(t, false), twi = to_wtw(t, true);
  int Ms[4];
  const int np = wave_plan(k, Ms);
  int lo[4];
  for (int i = 0, top = k; i < np; i++) { lo[i] = top - Ms[i]; top = lo[i]; }
  int rc;
  for (int i = 0; i < np - 1; i++) {
    const WPass p{k, lo[i]};
    rc = i == 0 ? fwd_m<R, true>(Ms[i], p, A, B, d_a, d_b, la, lb, twf, 2, st)
                : fwd_m<R, false>(Ms[i], p, A, B, nullptr, nullptr, 0, 0, twf, 2, st);
    if (rc) return rc;
  }
  const uint32_t tiles = (uint32_t)((1ull << k) >> WT_BITS);
  hipLaunchKernelGGL((wt_center_kernel<R>), dim3(tiles), dim3(Eng<R, WT_BITS>::NT), 0, st, WPass{k, 0}, A, B, twf,
                     twi);
  PLK_HIP(hipGetLastError());
  const uint64_t rl = la + lb - 1;
  for (int i = np - 2; i >= 0; i--) {
    const WPass p{k, lo[i]};
    rc = i == 0 ? inv_m<R, true>(Ms[i], p, A, twi, d_out, rl, ninv, st)
                : inv_m<R, false>(Ms[i], p, A, twi, nullptr, 0, 0u, st);
    if (rc) return rc;
  }
  return PLK_OK;
}

int plk_wave_poly_mul_launch(const uint8_t* d_a, uint64_t la, const uint8_t* d_b, uint64_t lb, int k,
                             uint8_t* d_out, uint32_t* A, uint32_t* B, uint32_t ninv, hipStream_t st) {
  switch (wt_radix_bits()) {
    case 3: return wave_poly_mul_r<3>(d_a, la, d_b, lb, k, d_out, A, B, ninv, st);
    case 4: return wave_poly_mul_r<4>(d_a, la, d_b, lb, k, d_out, A, B, ninv, st);
    default: return wave_poly_mul_r<2>(d_a, la, d_b, lb, k, d_out, A, B, ninv, st);
  }
}

template <int R>
static int wave_ntt_r(uint32_t* d, int k, int inverse, hipStream_t st) {
  const PlkTwTables t = plk_ntt_tables();
  int Ms[4];
  const int np = wave_plan(k, Ms);
  int lo[4];
  for (int i = 0, top = k; i < np; i++) { lo[i] = top - Ms[i]; top = lo[i]; }
  for (int s = 0; s < np; s++) {
    const int i = inverse ? np - 1 - s : s;
    const WPass p{k, lo[i]};
    const int rc = inverse ? inv_m<R, false>(Ms[i], p, d, to_wtw(t, true), nullptr, 0, 0u, st)
                           : fwd_m<R, false>(Ms[i], p, d, d, nullptr, nullptr, 0, 0, to_wtw(t, false), 1, st);
    if (rc) return rc;
  }
  return PLK_OK;
}

int plk_wave_ntt_launch(uint32_t* d, int k, int inverse, hipStream_t st) {
  switch (wt_radix_bits()) {
    case 3: return wave_ntt_r<3>(d, k, inverse, st);
    case 4: return wave_ntt_r<4>(d, k, inverse, st);
    default: return wave_ntt_r<2>(d, k, inverse, st);
  }
}
