// G1 multi-scalar multiplication for srs_eval_at_s (reference src/srs.h:53-68) on gfx950.
//
// The reference folds acc = acc + g1_mul(P_i, c_i) serially over GF(101) affine formulas
// (src/g1.h:37-103).  E(F101) is a cyclic group of order 102 and those formulas are an
// exact group law on it, so for canonical inputs the fold equals
//        EXP[ (sum_i c_i * LOG(P_i)) mod 102 ]
// with LOG/EXP the discrete-log tables of a generator g0 of order 102 (built on the host in
// capi.hip from the group law).  That turns the MSM into a one-pass, HBM-bound integer
// reduction: read 3 B of point + 1 B of scalar, one conflict-free LDS table read, a handful
// of VALU ops.  It is the degenerate case of Pippenger: a single 8-bit window whose
// "buckets" are the 102 group elements, accumulated as integers.
//
// Lookup: 101 = 2 mod 3, so cubing is a bijection of GF(101) and every y has exactly ONE x
// with y^2 = x^3 + 3.  A point is handled as k = (x << 8 | y << 16 | inf << 24) (one
// v_perm_b32 out of the loaded words) and looked up at idx = (y | (inf & 1) << 8):
//     E[y]        = X(y) << 8 | y << 16 | LOG(X(y), y)      y < 101 (the affine points)
//     E[256]      = 1 << 24                                   the identity {0, 0, 1}, log 0
//     E[other]    = a value whose y byte differs from idx's     never matches
// so d = E[idx] - k is the log (< 102) exactly when the encoding is canonical, and >= 256
// otherwise: one subtract, one compare, and the log feeds the multiply directly.  The
// table sits in LDS with 32 copies (copy = lane mod 32): the gathers are conflict free.
//
// Non-canonical encodings (off-curve points, coordinates >= 101, an infinite flag with
// coordinates, flag bytes other than 0/1) are not group elements; the reference still
// folds them with its raw formulas.  The kernel flags them and the host entry point re-runs
// the exact serial fold on the device (msm_serial_fold_kernel) -- bit-exact either way.
#include "plk_device.h"
#include "plk_internal.h"
#include "plk_msm_finish.h"

#include <stdlib.h>

#include <algorithm>

// Diagnostic builds only (tools/msm_lab.hip): bit 0 replaces the LDS table by arithmetic,
// bit 1 replaces the ticketed atomics by a plain store.  Always 0 in libplonkhip.
#ifndef PLK_MSM_DIAG
#define PLK_MSM_DIAG 0
#endif

__constant__ uint32_t c_ytab[512];             // E[idx], see above
__constant__ __attribute__((aligned(16))) uint8_t c_exp[PLK_GROUP_ORDER * 4];  // EXP[k] = {x, y, inf, 0}
__constant__ uint8_t c_inv101[PLK_GF_P];       // a^-1 mod 101 (0 -> 0), for the raw fold
__constant__ uint32_t c_inv101w[PLK_GF_P];     // the same as words (scalar loads in the uniform fold)
__device__ uint32_t g_exp_words[PLK_GROUP_ORDER];   // c_exp as words in global memory (plk_msm_exp_words_dev)

namespace {

// The table is kept in C copies (copy = lane mod C, entry-major: the C copies of an entry are
// consecutive words): more copies mean fewer bank conflicts in the gathers but a bigger
// per-block fill.  The launcher picks C per launch shape (plk_msm_geometry).
template <int C>
constexpr int copy_shift() { return C == 32 ? 7 : (C == 16 ? 6 : (C == 8 ? 5 : (C == 4 ? 4 : (C == 2 ? 3 : 2)))); }
constexpr int TAB_ENTRIES = 512;

// Encoded point j (0..15) of a 48-byte group held in w[0..11]: bytes 3j..3j+2 -> k = byte
// string shifted up by one byte (x << 8 | y << 16 | inf << 24).
template <int J>
__device__ __forceinline__ uint32_t point_bytes(const uint32_t (&w)[12]) {
  constexpr int o = 3 * J, d = o >> 2, b = o & 3;
  constexpr int d1 = (b + 2 <= 3) ? d : d + 1;
  // v_perm_b32: selector bytes 0-3 pick from the 2nd operand, 4-7 from the 1st, 0x0C -> 0
  constexpr uint32_t sel = 0x0Cu | ((uint32_t)b << 8) | ((uint32_t)(b + 1) << 16) | ((uint32_t)(b + 2) << 24);
  return __builtin_amdgcn_perm(w[d1], w[d], sel);
}

__device__ __forceinline__ uint32_t encode(uint32_t x, uint32_t y, uint32_t f) { return x << 8 | y << 16 | f << 24; }

// log(P) * c for one encoded point; flags non-canonical encodings in bad.  The product of
// a flagged point is garbage, which is fine: the result is then recomputed serially.
template <int C>
__device__ __forceinline__ uint32_t point_term(uint32_t k, uint32_t c, const uint32_t* tab, uint32_t lane4,
                                               bool& bad) {
  const uint32_t idx = (k >> 16) & 0x1FFu;
#if PLK_MSM_DIAG & 1
  const uint32_t e = idx * 0x9E37u + lane4;
#else
  const uint32_t e = *reinterpret_cast<const uint32_t*>(reinterpret_cast<const char*>(tab) + ((idx << copy_shift<C>()) | lane4));
#endif
  const uint32_t d = e - k;
  bad |= d >= 256u;
  return (d & 0xFFu) * c;
}

// Table fill in two halves so the caller can put the point loads between them: the table
// source words are loaded FIRST, the group loads after, and the LDS writes then wait with a
// counted vmcnt for the table words only (a fill loop that waits vmcnt(0) would also wait
// for the whole first group to arrive from HBM -- ~2 us per launch).
// C >= 4: uint4 stores of 4 copies of one entry; C < 4: one word store per (entry, copy).
template <int NT, int C>
struct TableFill {
  static constexpr int W = C >= 4 ? 4 : 1;                     // words per store
  static constexpr int STORES = TAB_ENTRIES * C / W;
  static constexpr int PER = (STORES + NT - 1) / NT;            // stores per thread
  uint32_t v[PER];
  __device__ __forceinline__ void load() {
#pragma unroll
    for (int j = 0; j < PER; j++) {
      const uint32_t i = threadIdx.x + j * NT;
      v[j] = c_ytab[(i * W / C) & (TAB_ENTRIES - 1)];
    }
  }
  __device__ __forceinline__ void store(uint32_t* tab) const {
#pragma unroll
    for (int j = 0; j < PER; j++) {
      const uint32_t i = threadIdx.x + j * NT;
      if (STORES % NT == 0 || i < STORES) {
        if (W == 4) reinterpret_cast<uint4*>(tab)[i] = make_uint4(v[j], v[j], v[j], v[j]);
        else tab[i] = v[j];
      }
    }
  }
};

struct Group {
  uint4 q0, q1, q2, s;
};

#ifndef PLK_MSM_NT
#define PLK_MSM_NT 0   // non-temporal (streaming) loads of the points and scalars (tuning)
#endif
typedef unsigned int plk_u32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ uint4 ld4(const uint4* p) {
  if (PLK_MSM_NT) {
    const plk_u32x4 v = __builtin_nontemporal_load(reinterpret_cast<const plk_u32x4*>(p));
    return make_uint4(v.x, v.y, v.z, v.w);
  }
  return *p;
}
__device__ __forceinline__ Group load_group(const uint4* p4, const uint4* s4, uint64_t g) {
  Group r;
  r.q0 = ld4(p4 + 3 * g + 0);
  r.q1 = ld4(p4 + 3 * g + 1);
  r.q2 = ld4(p4 + 3 * g + 2);
  r.s = ld4(s4 + g);
  return r;
}

template <int C, int J>
__device__ __forceinline__ void group_term(const uint32_t (&w)[12], const uint32_t (&sw)[4], const uint32_t* tab,
                                           uint32_t lane4, bool& bad, uint32_t& part) {
  part += point_term<C>(point_bytes<J>(w), (sw[J >> 2] >> (8 * (J & 3))) & 0xFFu, tab, lane4, bad);
}

template <int C>
__device__ __forceinline__ uint32_t group_sum(const Group& g, const uint32_t* tab, uint32_t lane4, bool& bad) {
  const uint32_t w[12] = {g.q0.x, g.q0.y, g.q0.z, g.q0.w, g.q1.x, g.q1.y, g.q1.z, g.q1.w,
                          g.q2.x, g.q2.y, g.q2.z, g.q2.w};
  const uint32_t sw[4] = {g.s.x, g.s.y, g.s.z, g.s.w};
  uint32_t part = 0;
  group_term<C, 0>(w, sw, tab, lane4, bad, part);   group_term<C, 1>(w, sw, tab, lane4, bad, part);
  group_term<C, 2>(w, sw, tab, lane4, bad, part);   group_term<C, 3>(w, sw, tab, lane4, bad, part);
  group_term<C, 4>(w, sw, tab, lane4, bad, part);   group_term<C, 5>(w, sw, tab, lane4, bad, part);
  group_term<C, 6>(w, sw, tab, lane4, bad, part);   group_term<C, 7>(w, sw, tab, lane4, bad, part);
  group_term<C, 8>(w, sw, tab, lane4, bad, part);   group_term<C, 9>(w, sw, tab, lane4, bad, part);
  group_term<C, 10>(w, sw, tab, lane4, bad, part);  group_term<C, 11>(w, sw, tab, lane4, bad, part);
  group_term<C, 12>(w, sw, tab, lane4, bad, part);  group_term<C, 13>(w, sw, tab, lane4, bad, part);
  group_term<C, 14>(w, sw, tab, lane4, bad, part);  group_term<C, 15>(w, sw, tab, lane4, bad, part);
  return part;                                   // <= 16 * 101 * 255
}

// Half a group (8 points, 24 B of points + 8 B of scalars) for one thread: the single-MSM
// form, where every thread has exactly one unit of work and the launch is ONE resident round.
// The terms are computed after the last word of the half arrives, so halving the work per
// thread (twice the waves) halves what the last-arriving waves still compute after the stream
// ends: a single 2^22-point MSM 0.2-0.3 us shorter (tools/msm_single_lab2.hip).
struct Half {
  uint2 a0, a1, a2, s;
};
__device__ __forceinline__ Half load_half(const uint8_t* pts, const uint8_t* sc, uint64_t u) {
  const uint2* pp = reinterpret_cast<const uint2*>(pts + 24 * u);   // 8-byte aligned: 48 (u/2) + 24 (u&1)
  Half h;
  h.a0 = pp[0];
  asm volatile("" ::: "memory");
  h.a1 = pp[1];
  asm volatile("" ::: "memory");
  h.a2 = pp[2];
  asm volatile("" ::: "memory");
  h.s = *reinterpret_cast<const uint2*>(sc + 8 * u);
  return h;
}
template <int C, int J>
__device__ __forceinline__ uint32_t half_d(const uint32_t (&w)[12], const uint32_t* tab, uint32_t lane4) {
  const uint32_t k = point_bytes<J>(w);
  const uint32_t idx = (k >> 16) & 0x1FFu;
  return *reinterpret_cast<const uint32_t*>(reinterpret_cast<const char*>(tab) + ((idx << copy_shift<C>()) | lane4)) - k;
}
// d = E - k per point (the log in byte 0 when canonical, >= 256 otherwise); the eight logs are
// packed two bytes at a time and multiplied by the scalar bytes with v_dot4_u32_u8.
template <int C>
__device__ __forceinline__ uint32_t half_sum(const Half& h, const uint32_t* tab, uint32_t lane4, bool& bad) {
  const uint32_t w[12] = {h.a0.x, h.a0.y, h.a1.x, h.a1.y, h.a2.x, h.a2.y, 0u, 0u, 0u, 0u, 0u, 0u};
  const uint32_t d0 = half_d<C, 0>(w, tab, lane4), d1 = half_d<C, 1>(w, tab, lane4);
  const uint32_t d2 = half_d<C, 2>(w, tab, lane4), d3 = half_d<C, 3>(w, tab, lane4);
  const uint32_t d4 = half_d<C, 4>(w, tab, lane4), d5 = half_d<C, 5>(w, tab, lane4);
  const uint32_t d6 = half_d<C, 6>(w, tab, lane4), d7 = half_d<C, 7>(w, tab, lane4);
  bad |= (d0 | d1 | d2 | d3 | d4 | d5 | d6 | d7) >= 256u;
  // perm selector 0x0C0C0400: byte 0 of the second operand, byte 0 of the first, zeros above
  const uint32_t lo = __builtin_amdgcn_perm(__builtin_amdgcn_perm(d3, d2, 0x0C0C0400u),
                                            __builtin_amdgcn_perm(d1, d0, 0x0C0C0400u), 0x05040100u);
  const uint32_t hi = __builtin_amdgcn_perm(__builtin_amdgcn_perm(d7, d6, 0x0C0C0400u),
                                            __builtin_amdgcn_perm(d5, d4, 0x0C0C0400u), 0x05040100u);
  return __builtin_amdgcn_udot4(hi, h.s.y, __builtin_amdgcn_udot4(lo, h.s.x, 0u, false), false);   // <= 8*101*255
}

}  // namespace

// One launch = a batch of gridDim.y MSMs of n points each (points/scalars of MSM b at
// pts + b * pstride, sc + b * sstride; result record res[b]); gridDim.x blocks per MSM,
// each striding over its MSM's 16-point groups, G groups in flight per thread.
//
// Finish without a second launch: every block reduces its points to a partial log (< 102)
// and adds   partial | 1 << 32 | (irregular ? 1 << 48 : 0)   with ONE 64-bit device-scope
// atomic to the shard word res[b].shard[s][0], s = (linear block id) mod 8 -- blocks are
// dealt round-robin over the 8 XCDs, so a shard is (for speed only) one XCD's blocks.  The
// shard words sit on separate 128-byte lines: device-scope atomics to one line serialise at
// ~10 ns each (256 arrivals on one word: +2.8 us per launch; 8 words on one line: no
// better; 8 lines: -1.7 us, tools/msm_lab.hip).  The block
// whose ticket comes back as (shard size - 1) owns the shard's complete sum (old + own add,
// no fence or re-read needed), re-arms the shard word and adds the shard total to
// res[b].top the same way; the last shard's finisher writes log / irregular / g1 and
// re-arms top.  Every word is zero again when the launch ends.
template <bool ALIGNED, int NT, int G, int COPIES, bool HALF>
__global__ __launch_bounds__(NT) void msm_dlog_kernel(const uint8_t* pts_base, uint64_t pstride,
                                                      const uint8_t* sc_base, uint64_t sstride,
                                                      uint64_t n, uint32_t full, PlkMsmResult* res_base) {
  __shared__ __attribute__((aligned(16))) uint32_t tab[TAB_ENTRIES * COPIES];
  __shared__ uint32_t etab[PLK_GROUP_ORDER];   // EXP words {x, y, inf, 0} for the last finisher
  __shared__ uint32_t wsum[NT / PLK_WAVE];
  __shared__ uint32_t wbad[NT / PLK_WAVE];
  const uint8_t* pts = pts_base + (uint64_t)blockIdx.y * pstride;
  const uint8_t* sc = sc_base + (uint64_t)blockIdx.y * sstride;
  PlkMsmResult* res = res_base + blockIdx.y;

  const uint64_t tid = (uint64_t)blockIdx.x * NT + threadIdx.x;
  const uint64_t stride = (uint64_t)gridDim.x * NT;
  const uint32_t lane4 = (threadIdx.x & (COPIES - 1u)) << 2;
  uint32_t acc = 0;
  bool bad = false;
  TableFill<NT, COPIES> fill;
  fill.load();                                  // table words first ...
  // ... with the EXP table (staged in LDS: the last finisher's point lookup is then not a
  // dependent global load at the very end of the launch, -0.15..0.3 us per single MSM)
  const uint32_t ev = threadIdx.x < PLK_GROUP_ORDER ? reinterpret_cast<const uint32_t*>(c_exp)[threadIdx.x] : 0u;

  const uint64_t ngroups = n >> 4;
  if (HALF) {
    // one resident round of half groups (8 points per thread, units of 24 B + 8 B); `full` is
    // unused: a thread takes units tid, tid + stride, ... (at most one in the launches that
    // use this form, see plk_msm_geometry)
    const uint64_t nunits = ngroups * 2;
    uint64_t u = tid;
    Half h{};
    asm volatile("" ::: "memory");
    if (u < nunits) h = load_half(pts, sc, u);
    if (!(PLK_MSM_DIAG & 1)) {
      fill.store(tab);
      if (threadIdx.x < PLK_GROUP_ORDER) etab[threadIdx.x] = ev;
      __syncthreads();
    }
    if (u < nunits) acc = half_sum<COPIES>(h, tab, lane4, bad) % PLK_GROUP_ORDER;
    for (u += stride; u < nunits; u += stride) acc += half_sum<COPIES>(load_half(pts, sc, u), tab, lane4, bad) % PLK_GROUP_ORDER;
    const uint64_t base = ngroups << 4;
    if (blockIdx.x == 0 && base + threadIdx.x < n) {
      const uint64_t i = base + threadIdx.x;
      acc += point_term<COPIES>(encode(pts[3 * i], pts[3 * i + 1], pts[3 * i + 2]), sc[i], tab, lane4, bad);
    }
  } else if (ALIGNED) {
    // 16 points per thread-step: 48 B of points (3 x dwordx4) + 16 B of scalars (1 x dwordx4)
    const uint4* p4 = reinterpret_cast<const uint4*>(pts);
    const uint4* s4 = reinterpret_cast<const uint4*>(sc);
    // `full` (from the host: ngroups / (stride G)) iterations in which every thread of the grid
    // has G groups, then one masked remainder step.  An iteration issues the loads of its G
    // groups (g, g + stride, ...) and then consumes them in issue order: no loaded register is
    // carried around the loop (a loop-carried prefetch makes the register allocator copy the
    // arrived group at the latch, i.e. wait for it), the compiler's vmcnt bookkeeping is exact
    // (vmcnt(4 (G-1-j)) before group j), and a group's lookups run while the later groups of
    // the same iteration are still arriving -- in a launch of one resident round (a single
    // MSM) that hides all but the last group's VALU work behind the stream.  The first
    // iteration is peeled so the table fill sits between its loads and its compute.
    const uint64_t span = stride * G;
    uint64_t g = tid;
    if (full > 0) {
      Group cur[G];
      asm volatile("" ::: "memory");
#pragma unroll
      for (int j = 0; j < G; j++) {
        cur[j] = load_group(p4, s4, g + j * stride);
        asm volatile("" ::: "memory");               // keep group j's loads older than j+1's
      }
      if (!(PLK_MSM_DIAG & 1)) {
        fill.store(tab);                              // ... LDS fill waits for the table words only
        if (threadIdx.x < PLK_GROUP_ORDER) etab[threadIdx.x] = ev;
        __syncthreads();
      }
      uint32_t part = 0;
#pragma unroll
      for (int j = 0; j < G; j++) part += group_sum<COPIES>(cur[j], tab, lane4, bad);
      acc = part % PLK_GROUP_ORDER;
      g += span;
    } else if (!(PLK_MSM_DIAG & 1)) {
      fill.store(tab);
      if (threadIdx.x < PLK_GROUP_ORDER) etab[threadIdx.x] = ev;
      __syncthreads();
    }
    for (uint32_t it = 1; it < full; it++, g += span) {
      Group cur[G];
      asm volatile("" ::: "memory");
#pragma unroll
      for (int j = 0; j < G; j++) {
        cur[j] = load_group(p4, s4, g + j * stride);
        asm volatile("" ::: "memory");
      }
      uint32_t part = 0;
#pragma unroll
      for (int j = 0; j < G; j++) part += group_sum<COPIES>(cur[j], tab, lane4, bad);
      acc += part % PLK_GROUP_ORDER;
    }
    // remainder: fewer than G groups per thread
#pragma unroll
    for (int j = 0; j < G; j++) {
      const uint64_t gj = g + j * stride;
      if (gj < ngroups) acc += group_sum<COPIES>(load_group(p4, s4, gj), tab, lane4, bad) % PLK_GROUP_ORDER;
    }
    // tail (n mod 16 points), one point per thread of the first block
    const uint64_t base = ngroups << 4;
    if (blockIdx.x == 0 && base + threadIdx.x < n) {
      const uint64_t i = base + threadIdx.x;
      acc += point_term<COPIES>(encode(pts[3 * i], pts[3 * i + 1], pts[3 * i + 2]), sc[i], tab, lane4, bad);
    }
  } else {
    fill.store(tab);
    if (threadIdx.x < PLK_GROUP_ORDER) etab[threadIdx.x] = ev;
    __syncthreads();
    for (uint64_t i = tid; i < n; i += stride) {
      acc += point_term<COPIES>(encode(pts[3 * i], pts[3 * i + 1], pts[3 * i + 2]), sc[i], tab, lane4, bad);
      acc %= PLK_GROUP_ORDER;
    }
  }
  acc %= PLK_GROUP_ORDER;
  msm_finish<NT>(acc, bad, res, wsum, wbad, etab);
}

// ---------------------------------------------------------------------------------------
// A FIXED SRS in log form.  The prover commits 9 polynomials against one SRS per proof
// (src/plonk.h:299-301, 379, 522-524, 620-621): it converts the SRS once (srs_log_kernel: LOG(P_i)
// as one byte, the same table lookup as above; any non-canonical encoding raises the flag and
// the caller keeps the G1 form), after which each commitment reads 1 B of log + 1 B of scalar
// per point instead of 3 + 1, and multiplies with v_dot4_u32_u8 (4 points per instruction).
// ---------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void srs_log_kernel(const uint8_t* __restrict__ pts, uint64_t n,
                                                      uint8_t* __restrict__ logs, uint32_t* __restrict__ irregular) {
  __shared__ uint32_t tab[TAB_ENTRIES];
  for (uint32_t i = threadIdx.x; i < TAB_ENTRIES; i += blockDim.x) tab[i] = c_ytab[i];
  __syncthreads();
  bool bad = false;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    const uint32_t k = encode(pts[3 * i], pts[3 * i + 1], pts[3 * i + 2]);
    const uint32_t d = tab[(k >> 16) & 0x1FFu] - k;
    bad |= d >= 256u;
    logs[i] = (uint8_t)d;
  }
  if (__ballot(bad) && (threadIdx.x & (PLK_WAVE - 1)) == 0) atomicOr(irregular, 1u);
}

// MSM b of the launch (b = blockIdx.y): logs at logs + b lstride, scalars at sc + b sstride, n
// points; 16-byte aligned bases (the caller checks).  Every thread takes 16-point groups with the
// grid's stride; the finish is msm_dlog_kernel's (msm_finish).
template <int NT>
__global__ __launch_bounds__(NT) void msm_log_kernel(const uint8_t* logs_base, uint64_t lstride, const uint8_t* sc_base,
                                                     uint64_t sstride, uint64_t n, PlkMsmResult* res_base) {
  __shared__ uint32_t etab[PLK_GROUP_ORDER];
  __shared__ uint32_t wsum[NT / PLK_WAVE];
  __shared__ uint32_t wbad[NT / PLK_WAVE];
  const uint8_t* lg = logs_base + (uint64_t)blockIdx.y * lstride;
  const uint8_t* sc = sc_base + (uint64_t)blockIdx.y * sstride;
  if (threadIdx.x < PLK_GROUP_ORDER) etab[threadIdx.x] = reinterpret_cast<const uint32_t*>(c_exp)[threadIdx.x];
  const uint64_t stride = (uint64_t)gridDim.x * NT;
  const uint64_t ngroups = n >> 4;
  const uint4* l4 = reinterpret_cast<const uint4*>(lg);
  const uint4* s4 = reinterpret_cast<const uint4*>(sc);
  uint32_t acc = 0;
  for (uint64_t g = (uint64_t)blockIdx.x * NT + threadIdx.x; g < ngroups; g += stride) {
    const uint4 a = l4[g], b = s4[g];
    uint32_t t = __builtin_amdgcn_udot4(a.x, b.x, 0u, false);   // 16 x 101 x 255 < 2^19
    t = __builtin_amdgcn_udot4(a.y, b.y, t, false);
    t = __builtin_amdgcn_udot4(a.z, b.z, t, false);
    t = __builtin_amdgcn_udot4(a.w, b.w, t, false);
    acc += t % PLK_GROUP_ORDER;
  }
  const uint64_t base = ngroups << 4;   // the n mod 16 tail: the first block
  if (blockIdx.x == 0 && base + threadIdx.x < n) acc += (uint32_t)lg[base + threadIdx.x] * sc[base + threadIdx.x];
  acc %= PLK_GROUP_ORDER;
  msm_finish<NT>(acc, false, res_base + blockIdx.y, wsum, wbad, etab);
}

// ---------------------------------------------------------------------------------------
// Exact serial fold on raw bytes, for inputs the discrete-log path flagged as irregular.
// Restates the reference arithmetic byte for byte (src/gf.h:87-162, src/g1.h:37-103):
// uint16 sums with one conditional subtract, int16 differences with one conditional add,
// products % 101, inverse a^99 (= INV[a mod 101] for a != 0 mod 101, 0 otherwise).
// ---------------------------------------------------------------------------------------
namespace {
struct RawPt { uint32_t x, y, inf; };

// inv: a^-1 mod 101 (0 -> 0), staged in LDS by the fold kernel for the per-lane term
// computation; nullptr: the __constant__ table (wave-uniform folding: scalar-cache loads)
struct RawOps {
  const uint32_t* inv;
  __device__ __forceinline__ uint32_t add(uint32_t a, uint32_t b) const { uint32_t s = a + b; return (s >= 101 ? s - 101 : s) & 0xFF; }
  __device__ __forceinline__ uint32_t sub(uint32_t a, uint32_t b) const { int d = (int)a - (int)b; if (d < 0) d += 101; return (uint32_t)d & 0xFF; }
  __device__ __forceinline__ uint32_t mul(uint32_t a, uint32_t b) const { return (a * b) % 101; }
  __device__ __forceinline__ uint32_t rinv(uint32_t a) const { return inv ? inv[a % 101] : c_inv101w[a % 101]; }
  __device__ __forceinline__ uint32_t red(uint32_t v) const { return v % 101; }  // f101(uint64 of a byte)

  __device__ RawPt dbl(RawPt a) const {
    if (a.inf || a.y == 0) return RawPt{0, 0, 1};
    const uint32_t m = mul(mul(3, mul(a.x, a.x)), rinv(mul(2, a.y)));
    const uint32_t m2 = mul(m, m);
    const uint32_t xr = sub(m2, mul(2, a.x));
    const uint32_t yr = sub(mul(m, sub(mul(3, a.x), m2)), a.y);
    return RawPt{red(xr), red(yr), 0};
  }
  __device__ RawPt addp(RawPt a, RawPt b) const {
    if (a.inf) return b;
    if (b.inf) return a;
    if (a.x == b.x) {
      if (add(a.y, b.y) == 0) return RawPt{0, 0, 1};
      return dbl(a);
    }
    const uint32_t m = mul(sub(b.y, a.y), rinv(sub(b.x, a.x)));
    const uint32_t xr = sub(sub(mul(m, m), a.x), b.x);
    const uint32_t yr = sub(mul(m, sub(a.x, xr)), a.y);
    return RawPt{red(xr), red(yr), 0};
  }
  // g1_mul (src/g1.h:91-103): LSB-first double-and-add over the scalar byte
  __device__ RawPt mulp(RawPt run, uint32_t k) const {
    RawPt term{0, 0, 1};
    for (; k; k >>= 1) {
      if (k & 1) term = addp(term, run);
      run = dbl(run);
    }
    return term;
  }
};
}  // namespace

// The reference's fold for inputs with irregular encodings, exactly.  For canonical points the
// raw formulas ARE the group law, so the fold's prefix up to the first irregular
// point equals EXP[sum c_i LOG(P_i)]: one block sums that prefix in parallel (discrete logs
// through the LDS table, 16 points per thread per chunk, stopping at the chunk that holds the
// first irregular point).  From that point on the fold is order-dependent: only the additions
// acc = acc + term_i are serial.  The terms g1_mul(P_i, c_i) are independent, so waves 1-15
// compute the next chunk of them into LDS while lane 0 of wave 0 folds the current chunk.
constexpr int FOLD_T = 1024, FOLD_E = 16, FOLD_CH = 4096;
__global__ __launch_bounds__(FOLD_T) void msm_serial_fold_kernel(const uint8_t* __restrict__ pts,
                                                                 const uint8_t* __restrict__ sc, uint64_t n,
                                                                 PlkMsmResult* res) {
  __shared__ uint32_t tab[TAB_ENTRIES];
  __shared__ uint32_t wsum[FOLD_T / PLK_WAVE];
  __shared__ uint32_t invl[PLK_GF_P];
  __shared__ uint32_t terms[2][FOLD_CH];   // packed x | y << 8 | inf << 16 (raw bytes)
  __shared__ unsigned long long s_first;
  if (blockIdx.x != 0) return;
  for (int i = threadIdx.x; i < TAB_ENTRIES; i += FOLD_T) tab[i] = c_ytab[i];
  for (int i = threadIdx.x; i < PLK_GF_P; i += FOLD_T) invl[i] = c_inv101[i];
  if (threadIdx.x == 0) s_first = ~0ull;
  __syncthreads();
  uint32_t acc = 0;
  uint64_t first = ~0ull;
  for (uint64_t base = 0; base < n && first == ~0ull; base += (uint64_t)FOLD_T * FOLD_E) {
    uint32_t lg[FOLD_E];
    unsigned long long mine = ~0ull;
#pragma unroll
    for (int k = 0; k < FOLD_E; k++) {
      const uint64_t i = base + (uint64_t)k * FOLD_T + threadIdx.x;
      lg[k] = 0;
      if (i < n) {
        bool bad = false;
        const uint32_t t = point_term<1>(encode(pts[3 * i], pts[3 * i + 1], pts[3 * i + 2]), sc[i], tab, 0u, bad);
        lg[k] = t;
        if (bad && i < mine) mine = i;
      }
    }
    if (mine != ~0ull) atomicMin(&s_first, mine);
    __syncthreads();
    first = s_first;                    // uniform: the first irregular index so far (or none)
#pragma unroll
    for (int k = 0; k < FOLD_E; k++) {
      const uint64_t i = base + (uint64_t)k * FOLD_T + threadIdx.x;
      if (i < first) acc += lg[k];      // (i < n: lg = 0 past the end)
    }
    acc %= PLK_GROUP_ORDER;
    __syncthreads();
  }
  const uint32_t ws = plk_wave_sum(acc);
  if ((threadIdx.x & (PLK_WAVE - 1)) == 0) wsum[threadIdx.x / PLK_WAVE] = ws;
  __syncthreads();
  // the fold over [0, first): every lane of wave 0 holds it (wave-uniform, scalar registers)
  RawPt a{0, 0, 1};
  if (threadIdx.x < PLK_WAVE) {
    uint32_t tot = 0;
    for (int w = 0; w < FOLD_T / PLK_WAVE; w++) tot += wsum[w];
    const uint32_t lg0 = (uint32_t)__builtin_amdgcn_readfirstlane((int)(tot % PLK_GROUP_ORDER));
    a = RawPt{c_exp[4 * lg0], c_exp[4 * lg0 + 1], c_exp[4 * lg0 + 2]};
  }
  const RawOps ops{invl};
  if (first < n) {                      // uniform
    auto fill = [&](uint32_t* buf, uint64_t base, uint32_t t0, uint32_t nt) {
      for (uint32_t j = t0; j < (uint32_t)FOLD_CH && base + j < n; j += nt) {
        const uint64_t i = base + j;
        const RawPt t = ops.mulp(RawPt{pts[3 * i], pts[3 * i + 1], pts[3 * i + 2]}, sc[i]);
        buf[j] = t.x | t.y << 8 | t.inf << 16;
      }
    };
    fill(terms[0], first, threadIdx.x, FOLD_T);
    __syncthreads();
    for (uint64_t c = 0;; c++) {
      const uint64_t base = first + c * FOLD_CH, next = base + FOLD_CH;
      if (threadIdx.x >= PLK_WAVE) {
        if (next < n) fill(terms[(c + 1) & 1], next, threadIdx.x - PLK_WAVE, FOLD_T - PLK_WAVE);
      } else {
        // wave 0 folds: 64 terms per LDS read (lane j holds term j), then term by term as
        // wave-uniform values -- the addition runs on the scalar unit, its inverses come from
        // the scalar cache (c_inv101)
        const uint32_t m = (uint32_t)(n - base < (uint64_t)FOLD_CH ? n - base : (uint64_t)FOLD_CH);
        const uint32_t* tb = terms[c & 1];
        const RawOps uni{nullptr};
        for (uint32_t j0 = 0; j0 < m; j0 += PLK_WAVE) {
          const uint32_t tv = j0 + threadIdx.x < m ? tb[j0 + threadIdx.x] : 0u;
          const uint32_t cnt = m - j0 < (uint32_t)PLK_WAVE ? m - j0 : (uint32_t)PLK_WAVE;
          for (uint32_t jj = 0; jj < cnt; jj++) {
            const uint32_t t = (uint32_t)__builtin_amdgcn_readlane((int)tv, (int)jj);
            // (a is the same in every lane: read as scalars, the addition's branches and
            // arithmetic stay on the scalar unit)
            const RawPt au{(uint32_t)__builtin_amdgcn_readfirstlane((int)a.x),
                           (uint32_t)__builtin_amdgcn_readfirstlane((int)a.y),
                           (uint32_t)__builtin_amdgcn_readfirstlane((int)a.inf)};
            a = uni.addp(au, RawPt{t & 0xFFu, (t >> 8) & 0xFFu, t >> 16});
          }
        }
      }
      __syncthreads();
      if (next >= n) break;
    }
  }
  if (threadIdx.x != 0) return;
  res->g1[0] = (uint8_t)a.x;
  res->g1[1] = (uint8_t)a.y;
  res->g1[2] = (uint8_t)a.inf;
  res->g1[3] = 0;
}

// ---------------------------------------------------------------------------------------
// The same fold for long inputs, in parallel over chunks (src/srs.h:59-66).
//
// Every g1_add result that is not an operand passed through is g1_new(x, y) -- reduced mod 101
// (src/g1.h:13-20, 55, 82) -- or the identity {0, 0, 1}.  So the accumulator is one of the
// 10,202 canonical states S = {(x, y, 0) : x, y < 101} + {identity}, except right after an
// operand passed through: acc = t when acc is "infinite" (or acc unchanged when t is), and then
// it may be a raw byte triple.  A chunk of terms is therefore a map S -> states, computed here
// for ALL 10,202 start states at once by one workgroup per chunk:
//   * trajectories that reach the same state merge (owner table, step-tagged atomicMax: the
//     lowest trajectory id wins, the others record it as parent);
//   * trajectories on group elements (canonical on-curve points and the identity: the
//     reference's formulas ARE the group law there) are kept symbolically in a
//     102-slot table indexed by log - delta, and a regular term (a canonical group element of
//     log l) costs delta += l for all of them; an irregular term materialises them first;
//   * at most two raw trajectories exist at once (a raw state only arises as the current term
//     or survives an infinite term), kept in a side list and merged by exact bytes.
// Random chunk maps collapse fast: 10,202 start states -> ~500 live trajectories after 256
// terms, to the group (regular terms) or to a handful (irregular ones) after ~1000.  A
// single-wave pass then walks the chunk maps in order from the prefix state (one dependent
// load per chunk), re-folding a chunk serially only when a raw state crosses its boundary.
// ---------------------------------------------------------------------------------------
namespace {
constexpr int FS_N = 10202;                  // canonical states: x * 101 + y (inf 0), FS_ID = identity
constexpr int FS_ID = 10201;
constexpr uint32_t FS_EMPTY = 0xFFFFu;
constexpr int FC_T = 1024;                   // threads of a chunk workgroup
constexpr int FC_TB = 1024;                  // terms staged in LDS per refill
constexpr int FC_SOLO = 512;                 // live trajectories at which wave 0 continues alone
constexpr uint32_t FC_HDR_BYTES = 256;

struct FoldHdr {
  unsigned long long first;                  // first irregular point (n if none)
  uint32_t plog;                             // log of the fold over [0, first)
};

__device__ __forceinline__ uint32_t pk(RawPt a) { return a.x | a.y << 8 | a.inf << 16; }
__device__ __forceinline__ RawPt upk(uint32_t v) { return RawPt{v & 0xFFu, (v >> 8) & 0xFFu, (v >> 16) & 0xFFu}; }
__device__ __forceinline__ RawPt state_of(uint32_t id) {
  return id == FS_ID ? RawPt{0, 0, 1} : RawPt{id / 101u, id % 101u, 0};
}
__device__ __forceinline__ int id_of(RawPt a) {
  if (a.inf == 0 && a.x < 101 && a.y < 101) return (int)(a.x * 101 + a.y);
  return (a.inf == 1 && a.x == 0 && a.y == 0) ? FS_ID : -1;
}
// log of a canonical group element encoding, 0xFF for anything else (ytab: the dlog table)
__device__ __forceinline__ uint32_t glog(RawPt a, const uint32_t* ytab) {
  const uint32_t k = encode(a.x, a.y, a.inf);
  const uint32_t d = ytab[(a.y | (a.inf & 1u) << 8) & 0x1FFu] - k;
  return d < 256u ? d : 0xFFu;
}
}  // namespace

// Prefix: the fold over [0, first) -- all canonical points -- as a discrete-log sum, and the
// first irregular point (one block; every point read once).
__global__ __launch_bounds__(FOLD_T) void msm_fold_prefix_kernel(const uint8_t* __restrict__ pts,
                                                                 const uint8_t* __restrict__ sc, uint64_t n,
                                                                 FoldHdr* hdr) {
  __shared__ uint32_t tab[TAB_ENTRIES];
  __shared__ uint32_t wsum[FOLD_T / PLK_WAVE];
  __shared__ unsigned long long s_first;
  for (int i = threadIdx.x; i < TAB_ENTRIES; i += FOLD_T) tab[i] = c_ytab[i];
  if (threadIdx.x == 0) s_first = ~0ull;
  __syncthreads();
  uint32_t acc = 0;
  uint64_t first = ~0ull;
  for (uint64_t base = 0; base < n && first == ~0ull; base += (uint64_t)FOLD_T * FOLD_E) {
    uint32_t lg[FOLD_E];
    unsigned long long mine = ~0ull;
#pragma unroll
    for (int k = 0; k < FOLD_E; k++) {
      const uint64_t i = base + (uint64_t)k * FOLD_T + threadIdx.x;
      lg[k] = 0;
      if (i < n) {
        bool bad = false;
        lg[k] = point_term<1>(encode(pts[3 * i], pts[3 * i + 1], pts[3 * i + 2]), sc[i], tab, 0u, bad);
        if (bad && i < mine) mine = i;
      }
    }
    if (mine != ~0ull) atomicMin(&s_first, mine);
    __syncthreads();
    first = s_first;
#pragma unroll
    for (int k = 0; k < FOLD_E; k++) {
      const uint64_t i = base + (uint64_t)k * FOLD_T + threadIdx.x;
      if (i < first) acc += lg[k];
    }
    acc %= PLK_GROUP_ORDER;
    __syncthreads();
  }
  const uint32_t ws = plk_wave_sum(acc);
  if ((threadIdx.x & (PLK_WAVE - 1)) == 0) wsum[threadIdx.x / PLK_WAVE] = ws;
  __syncthreads();
  if (threadIdx.x == 0) {
    uint32_t tot = 0;
    for (int w = 0; w < FOLD_T / PLK_WAVE; w++) tot += wsum[w];
    hdr->first = first < n ? first : n;
    hdr->plog = tot % PLK_GROUP_ORDER;
  }
}

// One chunk [first + b L, first + (b + 1) L) per workgroup: F[b * FS_N + s] = the packed state
// the chunk's terms take start state s to.
__global__ __launch_bounds__(FC_T) void msm_fold_chunk_kernel(const uint8_t* __restrict__ pts,
                                                              const uint8_t* __restrict__ sc, uint64_t n,
                                                              uint32_t L, const FoldHdr* __restrict__ hdr,
                                                              uint32_t* __restrict__ F) {
  __shared__ uint32_t owner[FS_N];           // step-tagged claims; at the end: final state per trajectory
  __shared__ uint32_t lst[2][FS_N];          // concrete trajectories: state id | trajectory id << 14
  __shared__ uint16_t par[FS_N];             // merge parent (self = live)
  __shared__ uint32_t ytab[TAB_ENTRIES];
  __shared__ uint32_t invl[PLK_GF_P];
  __shared__ uint32_t expw[PLK_GROUP_ORDER]; // EXP as packed bytes
  __shared__ uint32_t gslot[PLK_GROUP_ORDER];
  __shared__ uint32_t tt[FC_TB];             // term bytes | log << 24 (log 0xFF: irregular)
  __shared__ uint32_t rawst[8], rawtid[8], stst[16], sttid[16];
  __shared__ uint32_t s_cnt[4], s_ng, s_nr, s_ns;
  const uint64_t first = hdr->first;
  const uint64_t c0 = first + (uint64_t)blockIdx.x * L;
  if (c0 >= n) return;
  const uint64_t c1 = n - c0 < L ? n : c0 + L;
  const uint32_t me = threadIdx.x;
  uint32_t nt = FC_T;
  for (uint32_t i = me; i < TAB_ENTRIES; i += nt) ytab[i] = c_ytab[i];
  for (uint32_t i = me; i < PLK_GF_P; i += nt) invl[i] = c_inv101[i];
  for (uint32_t i = me; i < PLK_GROUP_ORDER; i += nt)
    expw[i] = c_exp[4 * i] | (uint32_t)c_exp[4 * i + 1] << 8 | (uint32_t)c_exp[4 * i + 2] << 16;
  if (me < 2) s_cnt[me] = 0;
  if (me == 0) { s_ng = PLK_GROUP_ORDER; s_nr = 0; s_ns = 0; }
  __syncthreads();
  const RawOps ops{invl};
  for (uint32_t i = me; i < FS_N; i += nt) {
    owner[i] = 0;
    par[i] = (uint16_t)i;
    const RawPt a = state_of(i);
    const uint32_t lg = glog(a, ytab);
    if (lg < PLK_GROUP_ORDER) gslot[lg] = i;            // delta = 0: slot = log
    else lst[0][atomicAdd(&s_cnt[0], 1u)] = i | i << 14;
  }
  __syncthreads();
  // block-wide barriers while many trajectories are live; once few are, wave 0 continues alone
  // with wave-level ordering of its LDS traffic (the other waves wait at the barrier after the
  // loop, so every barrier is reached by every wave)
  bool solo = false;
  auto sync = [&]() {
    if (solo) {
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
    } else {
      __syncthreads();
    }
  };
  uint32_t cur = 0, delta = 0, step = 1;
  for (uint64_t i = c0; i < c1; i++, step++) {
    const uint32_t k = (uint32_t)((i - c0) % FC_TB);
    if (k == 0) {            // stage the next terms: g1_mul(P_i, c_i) on raw bytes, and their logs
      sync();
      for (uint32_t j = me; j < FC_TB && i + j < c1; j += nt) {
        const uint64_t q = i + j;
        const RawPt t = ops.mulp(RawPt{pts[3 * q], pts[3 * q + 1], pts[3 * q + 2]}, sc[q]);
        tt[j] = pk(t) | glog(t, ytab) << 24;
      }
      sync();
    }
    const uint32_t tv = tt[k];
    const uint32_t tl = tv >> 24;
    const RawPt t = upk(tv);
    uint32_t nc = s_cnt[cur];
    const uint32_t nr = s_nr;
    if (tl < PLK_GROUP_ORDER) {
      delta += tl;
      if (delta >= PLK_GROUP_ORDER) delta -= PLK_GROUP_ORDER;
    } else if (s_ng) {       // an irregular term: the symbolic group trajectories become concrete
      for (uint32_t r = me; r < PLK_GROUP_ORDER; r += nt) {   // (nt = 64 once wave 0 is alone)
        const uint32_t g = gslot[r];
        if (g != FS_EMPTY) {
          uint32_t e = r + delta;
          if (e >= PLK_GROUP_ORDER) e -= PLK_GROUP_ORDER;
          lst[cur][atomicAdd(&s_cnt[cur], 1u)] = (uint32_t)id_of(upk(expw[e])) | g << 14;
          gslot[r] = FS_EMPTY;
        }
      }
      sync();
      if (me == 0) s_ng = 0;
      nc = s_cnt[cur];
    }
    if (nc == 0 && nr == 0) continue;
    // pass 1: apply the term; claim the resulting canonical states
    for (uint32_t e = me; e < nc + nr; e += nt) {
      uint32_t tid;
      RawPt a;
      if (e < nc) {
        const uint32_t w = lst[cur][e];
        tid = w >> 14;
        a = state_of(w & 0x3FFFu);
      } else {
        tid = rawtid[e - nc];
        a = upk(rawst[e - nc]);
      }
      const RawPt b = ops.addp(a, t);
      const int s2 = id_of(b);
      if (s2 >= 0) {
        atomicMax(&owner[s2], step << 16 | (0xFFFFu - tid));
        lst[cur][e] = (uint32_t)s2 | tid << 14;
      } else {
        const uint32_t j = atomicAdd(&s_ns, 1u);
        if (j < 16) { stst[j] = pk(b); sttid[j] = tid; }
        lst[cur][e] = ~0u;
      }
    }
    sync();
    // pass 2: losers merge into the owner; owners on group elements join the symbolic slots,
    // the others go to the next list; raw results merge by bytes
    if (me == 0) {
      const uint32_t ns = s_ns < 16 ? s_ns : 16;
      uint32_t kept = 0;
      for (uint32_t j = 0; j < ns; j++) {
        uint32_t q = 0;
        while (q < kept && rawst[q] != stst[j]) q++;
        if (q < kept) par[sttid[j]] = (uint16_t)rawtid[q];
        else { rawst[kept] = stst[j]; rawtid[kept] = sttid[j]; kept++; }
      }
      s_nr = kept;
      s_ns = 0;
      s_cnt[cur] = 0;        // (this list is refilled by the next step's pass 2)
    }
    for (uint32_t e = me; e < nc + nr; e += nt) {
      const uint32_t w = lst[cur][e];
      if (w == ~0u) continue;
      const uint32_t s2 = w & 0x3FFFu, tid = w >> 14;
      const uint32_t win = 0xFFFFu - (owner[s2] & 0xFFFFu);
      if (win != tid) { par[tid] = (uint16_t)win; continue; }
      const uint32_t lg = glog(state_of(s2), ytab);
      if (lg < PLK_GROUP_ORDER) {
        const uint32_t r = lg >= delta ? lg - delta : lg + PLK_GROUP_ORDER - delta;
        const uint32_t occ = gslot[r];
        if (occ != FS_EMPTY) par[tid] = (uint16_t)occ;
        else { gslot[r] = tid; atomicAdd(&s_ng, 1u); }
      } else {
        lst[cur ^ 1][atomicAdd(&s_cnt[cur ^ 1], 1u)] = w;
      }
    }
    sync();
    cur ^= 1;
    if (!solo) {
      // every wave reads the counts before wave 0 can change them again (the next step's
      // materialisation appends before its first barrier): the decision is uniform
      const bool few = s_cnt[cur] + s_ng + s_nr <= FC_SOLO;
      __syncthreads();
      if (few) {
        if (me >= PLK_WAVE) break;
        solo = true;
        nt = PLK_WAVE;
      }
    }
  }
  __syncthreads();
  nt = FC_T;
  // (every wave: cur and delta as wave 0 left them)
  if (me == 0) { s_cnt[2 + 0] = cur; s_cnt[2 + 1] = delta; }
  __syncthreads();
  cur = s_cnt[2];
  delta = s_cnt[3];
  // final state of every live trajectory (owner reused), then every start state through its parents
  const uint32_t nc = s_cnt[cur], nr = s_nr;
  for (uint32_t e = me; e < nc; e += nt) {
    const uint32_t w = lst[cur][e];
    owner[w >> 14] = pk(state_of(w & 0x3FFFu));
  }
  for (uint32_t r = me; r < PLK_GROUP_ORDER; r += nt)
    if (gslot[r] != FS_EMPTY) owner[gslot[r]] = expw[r + delta < PLK_GROUP_ORDER ? r + delta : r + delta - PLK_GROUP_ORDER];
  for (uint32_t e = me; e < nr; e += nt) owner[rawtid[e]] = rawst[e];
  __syncthreads();
  uint32_t* out = F + (size_t)blockIdx.x * FS_N;
  for (uint32_t s0 = me; s0 < FS_N; s0 += nt) {
    uint32_t r = s0;
    while (par[r] != r) r = par[r];
    out[s0] = owner[r];
  }
}

// The chunk maps in order from the prefix state; a raw state at a chunk boundary re-folds that
// chunk serially (one wave: terms by lane, the additions wave-uniform).
__global__ __launch_bounds__(PLK_WAVE) void msm_fold_resolve_kernel(const uint8_t* __restrict__ pts,
                                                                    const uint8_t* __restrict__ sc, uint64_t n,
                                                                    uint32_t L, const FoldHdr* __restrict__ hdr,
                                                                    const uint32_t* __restrict__ F, PlkMsmResult* res) {
  __shared__ uint32_t invl[PLK_GF_P];
  for (int i = threadIdx.x; i < PLK_GF_P; i += PLK_WAVE) invl[i] = c_inv101[i];
  __syncthreads();
  const uint64_t first = hdr->first;
  const uint32_t pl = hdr->plog;
  uint32_t st = c_exp[4 * pl] | (uint32_t)c_exp[4 * pl + 1] << 8 | (uint32_t)c_exp[4 * pl + 2] << 16;
  const RawOps ops{invl}, uni{nullptr};
  for (uint64_t c0 = first, b = 0; c0 < n; c0 += L, b++) {
    const int id = id_of(upk(st));
    if (id >= 0) {
      st = (uint32_t)__builtin_amdgcn_readfirstlane((int)F[b * FS_N + (uint32_t)id]);
      continue;
    }
    const uint64_t c1 = n - c0 < L ? n : c0 + L;
    RawPt a = upk(st);
    for (uint64_t j0 = c0; j0 < c1; j0 += PLK_WAVE) {
      const uint64_t q = j0 + threadIdx.x;
      const uint32_t tv = q < c1 ? pk(ops.mulp(RawPt{pts[3 * q], pts[3 * q + 1], pts[3 * q + 2]}, sc[q])) : 0u;
      const uint32_t cnt = c1 - j0 < (uint64_t)PLK_WAVE ? (uint32_t)(c1 - j0) : (uint32_t)PLK_WAVE;
      for (uint32_t jj = 0; jj < cnt; jj++) {
        const RawPt au{(uint32_t)__builtin_amdgcn_readfirstlane((int)a.x), (uint32_t)__builtin_amdgcn_readfirstlane((int)a.y),
                       (uint32_t)__builtin_amdgcn_readfirstlane((int)a.inf)};
        a = uni.addp(au, upk((uint32_t)__builtin_amdgcn_readlane((int)tv, (int)jj)));
      }
    }
    st = pk(a);
  }
  if (threadIdx.x != 0) return;
  res->g1[0] = (uint8_t)(st & 0xFFu);
  res->g1[1] = (uint8_t)((st >> 8) & 0xFFu);
  res->g1[2] = (uint8_t)((st >> 16) & 0xFFu);
  res->g1[3] = 0;
}

// Combine per-shard partial logs (e.g. after an RCCL all-reduce SUM of int32 logs) into
// the final point: out = EXP[sum mod 102].
__global__ void msm_combine_kernel(const uint32_t* __restrict__ logs, int count, uint8_t* out) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  uint64_t s = 0;
  for (int i = 0; i < count; i++) s += logs[i];
  const uint32_t lg = (uint32_t)(s % PLK_GROUP_ORDER);
  out[0] = c_exp[4 * lg + 0];
  out[1] = c_exp[4 * lg + 1];
  out[2] = c_exp[4 * lg + 2];
}

// Batched finalisation: out[4 i .. 4 i + 3] = EXP[logs[i * stride] mod 102] for i < batch.
// Used after a collective SUM of per-rank partial logs for a batch of MSMs.
__global__ void msm_finalize_kernel(const uint32_t* __restrict__ logs, int batch, int stride, uint8_t* out) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= batch) return;
  const uint32_t lg = logs[(int64_t)i * stride] % PLK_GROUP_ORDER;
  out[4 * i + 0] = c_exp[4 * lg + 0];
  out[4 * i + 1] = c_exp[4 * lg + 1];
  out[4 * i + 2] = c_exp[4 * lg + 2];
  out[4 * i + 3] = 0;
}

// ------------------------------------------------------------------------------ launchers
int plk_msm_upload_tables(const uint32_t* ytab, const uint8_t* exp4, const uint8_t* inv101) {
  PLK_HIP(hipMemcpyToSymbol(HIP_SYMBOL(c_ytab), ytab, sizeof(uint32_t) * 512));
  PLK_HIP(hipMemcpyToSymbol(HIP_SYMBOL(c_exp), exp4, PLK_GROUP_ORDER * 4));
  PLK_HIP(hipMemcpyToSymbol(HIP_SYMBOL(c_inv101), inv101, PLK_GF_P));
  uint32_t w[PLK_GF_P];
  for (int i = 0; i < PLK_GF_P; i++) w[i] = inv101[i];
  PLK_HIP(hipMemcpyToSymbol(HIP_SYMBOL(c_inv101w), w, sizeof w));
  PLK_HIP(hipMemcpyToSymbol(HIP_SYMBOL(g_exp_words), exp4, PLK_GROUP_ORDER * 4));
  return PLK_OK;
}

const uint32_t* plk_msm_exp_words_dev() {   // (the current device's copy)
  void* p = nullptr;
  return hipGetSymbolAddress(&p, HIP_SYMBOL(g_exp_words)) == hipSuccess ? (const uint32_t*)p : nullptr;
}

// Launch geometry.  Big MSMs use 512-thread blocks (two 64 KB tables per CU, 16 waves);
// small ones 256-thread blocks so they still spread over many CUs.  Blocks per MSM:
//   * at least enough to fill the chip once (512 resident blocks shared by the batch), at
//     most one 16-point group per thread;
//   * and no fewer than one block per 2 groups per thread (32 points, 64 KB of input per
//     512-thread block -- the size of its LDS table).
// For large batches the second bound wins and the launch runs many rounds of short blocks:
// the chip then sweeps a few MSMs at a time instead of every block of one resident round
// striding through all of them, and blocks that finish early take more work.  Measured at
// 40 x 2^22 points per launch: 480 blocks 120 us, 10240 blocks 105 us (6.4 TB/s);
// at 8 x 2^22: 25.3 -> 24.9 us; one MSM: unchanged (tools/msm_layout_lab.hip).
// G (groups in flight per thread and iteration) is 1: with <= 2 groups per thread two
// iterations of one group measured faster than one of two.
// Overridable for tuning with PLK_OPT_MSM_THREADS / _MAX_BLOCKS / _GROUPS / _COPIES / _HALF.
void plk_msm_geometry(uint64_t n, int batch, int* threads, int* blocks, int* gpt, int* copies, int* half) {
  const int env_threads = (int)plk_opt(PLK_OPT_MSM_THREADS), env_blocks = (int)plk_opt(PLK_OPT_MSM_MAX_BLOCKS),
            env_g = (int)plk_opt(PLK_OPT_MSM_GROUPS), env_c = (int)plk_opt(PLK_OPT_MSM_COPIES),
            env_half = (int)plk_opt(PLK_OPT_MSM_HALF);
  const uint64_t groups = n >> 4;
  int th = groups >= 64ull * 1024 ? 512 : 256;
  if (env_threads == 256 || env_threads == 512 || env_threads == 1024) th = env_threads;
  uint64_t fill = env_blocks > 0 ? (uint64_t)env_blocks : 512;           // resident blocks
  fill = fill / (uint64_t)batch > 1 ? fill / (uint64_t)batch : 1;
  const uint64_t one_per_thread = (groups + th - 1) / th;
  const uint64_t two_per_thread = (groups + 2 * (uint64_t)th - 1) / (2 * (uint64_t)th);
  uint64_t b = fill < one_per_thread ? fill : one_per_thread;
  // batches: one group per thread (twice the blocks of two per thread: 160 x 2^22 points per
  // launch 0.787-0.790 -> 0.803-0.805 of 8 TB/s, same box, alternating); a single MSM keeps two
  if (env_blocks <= 0 && two_per_thread > b) b = batch >= 2 ? one_per_thread : two_per_thread;
  if (b < 1) b = 1;
  if (b > 8ull * 65535ull) b = 8ull * 65535ull;   // the finish's per-shard ticket field is 16 bits
  const uint64_t per_thread = groups / (b * (uint64_t)th);
  int g = 1;
  // two groups in flight per thread where a thread has them (with the 16 KB table four blocks
  // share a CU; +1.5-2 % on the headline over one group; PLK_OPT_MSM_GROUPS overrides)
  const int gmax = (env_g == 1 || env_g == 2 || env_g == 4) ? env_g : 2;
  while (g < gmax && (uint64_t)(2 * g) <= per_thread) g *= 2;
  // table copies: eight keep the gathers nearly conflict-free (a single 2^22-point MSM: lookups
  // 0.2 us shorter than with one copy, tools/msm_single_lab.hip) and the fill is off the
  // critical path (its words are loaded before the points); PLK_OPT_MSM_COPIES = 1 for tuning
  int c = 8;
  if (env_c == 1 || env_c == 8) c = env_c;
  // a single MSM whose threads have at most one group each (one resident round): half groups
  // on twice the blocks, one table copy (lab: the smaller fill wins there, 0.05-0.2 us)
  int hf = 0;
  if (env_half && batch == 1 && groups <= b * (uint64_t)th && 2 * b <= 8ull * 65535ull) {
    hf = 1;
    b *= 2;
    g = 1;
    c = env_c == 8 ? 8 : 1;
  }
  *threads = th;
  *blocks = (int)b;
  if (gpt) *gpt = g;
  if (copies) *copies = c;
  if (half) *half = hf;
}

namespace {
template <bool A, int T, int C>
void go_g(int g, dim3 grid, hipStream_t st, const uint8_t* p, uint64_t ps, const uint8_t* s, uint64_t ss, uint64_t n,
          PlkMsmResult* r) {
  if (!A) g = 1;
  const uint64_t span = (uint64_t)grid.x * T * g;
  const uint32_t full = (uint32_t)((n >> 4) / span);
  if (g == 1)
    hipLaunchKernelGGL((msm_dlog_kernel<A, T, 1, C, false>), grid, dim3(T), 0, st, p, ps, s, ss, n, full, r);
  else if (g == 2)
    hipLaunchKernelGGL((msm_dlog_kernel<A, T, 2, C, false>), grid, dim3(T), 0, st, p, ps, s, ss, n, full, r);
  else
    hipLaunchKernelGGL((msm_dlog_kernel<A, T, 4, C, false>), grid, dim3(T), 0, st, p, ps, s, ss, n, full, r);
}
template <int T>
void go_t(bool aligned, int g, int c, int half, dim3 grid, hipStream_t st, const uint8_t* p, uint64_t ps,
          const uint8_t* s, uint64_t ss, uint64_t n, PlkMsmResult* r) {
  if (aligned && half) {
    if (c == 1) hipLaunchKernelGGL((msm_dlog_kernel<true, T, 1, 1, true>), grid, dim3(T), 0, st, p, ps, s, ss, n, 0u, r);
    else hipLaunchKernelGGL((msm_dlog_kernel<true, T, 1, 8, true>), grid, dim3(T), 0, st, p, ps, s, ss, n, 0u, r);
  } else if (aligned) {
    if (c == 1) go_g<true, T, 1>(g, grid, st, p, ps, s, ss, n, r);
    else go_g<true, T, 8>(g, grid, st, p, ps, s, ss, n, r);
  } else {
    if (c == 1) go_g<false, T, 1>(g, grid, st, p, ps, s, ss, n, r);
    else go_g<false, T, 8>(g, grid, st, p, ps, s, ss, n, r);
  }
}
}  // namespace

int plk_msm_batch_launch(const uint8_t* d_pts, uint64_t pstride, const uint8_t* d_sc, uint64_t sstride, uint64_t n,
                         int batch, PlkMsmResult* d_res, hipStream_t st) {
  if (batch <= 0) return PLK_OK;
  if (batch > 65535) {
    plk_set_error("plk_msm batch %d too large", batch);
    return PLK_ERR_RANGE;
  }
  int threads, blocks, g, c, half;
  plk_msm_geometry(n, batch, &threads, &blocks, &g, &c, &half);
  const bool aligned = ((uintptr_t)d_pts % 16 == 0) && ((uintptr_t)d_sc % 16 == 0) &&
                       (batch == 1 || (pstride % 16 == 0 && sstride % 16 == 0));
  if (!aligned && half) {   // the byte-wise form: the plain plan
    half = 0;
    blocks /= 2;
  }
  const dim3 grid(blocks, batch);
  if (threads == 1024) go_t<1024>(aligned, g, c, half, grid, st, d_pts, pstride, d_sc, sstride, n, d_res);
  else if (threads == 512) go_t<512>(aligned, g, c, half, grid, st, d_pts, pstride, d_sc, sstride, n, d_res);
  else go_t<256>(aligned, g, c, half, grid, st, d_pts, pstride, d_sc, sstride, n, d_res);
  PLK_HIP(hipGetLastError());
  return PLK_OK;
}

int plk_msm_launch(const uint8_t* d_pts, const uint8_t* d_sc, uint64_t n, PlkMsmResult* d_res, hipStream_t st) {
  return plk_msm_batch_launch(d_pts, 0, d_sc, 0, n, 1, d_res, st);
}

// The exact raw fold (src/srs.h:59-66) for inputs with irregular encodings.  Short inputs: one
// block (parallel canonical prefix, then the serial additions).  Long ones: the chunk maps
// (msm_fold_*_kernel), whose scratch -- the chunk maps, 40.8 KB per chunk -- is stream-ordered
// (hipMallocAsync / hipFreeAsync on the caller's stream).
constexpr uint64_t FOLD_CHUNKED_MIN = 8192;
int plk_msm_serial_launch(const uint8_t* d_pts, const uint8_t* d_sc, uint64_t n, PlkMsmResult* d_res,
                          hipStream_t st) {
  if (n < FOLD_CHUNKED_MIN) {
    hipLaunchKernelGGL(msm_serial_fold_kernel, dim3(1), dim3(FOLD_T), 0, st, d_pts, d_sc, n, d_res);
    PLK_HIP(hipGetLastError());
    return PLK_OK;
  }
  // about one chunk per CU (one 150 KB workgroup each), 2048 .. 32768 terms per chunk
  uint64_t L = (n + 255) / 256;
  L = (L + 1023) & ~1023ull;
  L = L < 2048 ? 2048 : (L > 32768 ? 32768 : L);
  const uint64_t nch = (n + L - 1) / L;
  const size_t ws = FC_HDR_BYTES + (size_t)nch * FS_N * 4;
  void* w = nullptr;
  PLK_HIP(hipMallocAsync(&w, ws, st));
  FoldHdr* hdr = (FoldHdr*)w;
  uint32_t* F = (uint32_t*)((uint8_t*)w + FC_HDR_BYTES);
  hipLaunchKernelGGL(msm_fold_prefix_kernel, dim3(1), dim3(FOLD_T), 0, st, d_pts, d_sc, n, hdr);
  hipLaunchKernelGGL(msm_fold_chunk_kernel, dim3((unsigned)nch), dim3(FC_T), 0, st, d_pts, d_sc, n, (uint32_t)L, hdr, F);
  hipLaunchKernelGGL(msm_fold_resolve_kernel, dim3(1), dim3(PLK_WAVE), 0, st, d_pts, d_sc, n, (uint32_t)L, hdr, F,
                     d_res);
  const hipError_t le = hipGetLastError();
  PLK_HIP(hipFreeAsync(w, st));
  PLK_HIP(le);
  return PLK_OK;
}

int plk_msm_finalize_launch(const uint32_t* d_logs, int batch, int stride, uint8_t* d_out, hipStream_t st) {
  if (batch <= 0) return PLK_OK;
  hipLaunchKernelGGL(msm_finalize_kernel, dim3((batch + 255) / 256), dim3(256), 0, st, d_logs, batch, stride, d_out);
  PLK_HIP(hipGetLastError());
  return PLK_OK;
}

int plk_msm_combine_launch(const uint32_t* d_logs, int count, uint8_t* d_out, hipStream_t st) {
  hipLaunchKernelGGL(msm_combine_kernel, dim3(1), dim3(64), 0, st, d_logs, count, d_out);
  PLK_HIP(hipGetLastError());
  return PLK_OK;
}

int plk_srs_log_launch(const uint8_t* d_pts, uint64_t n, uint8_t* d_logs, uint32_t* d_irregular, hipStream_t st) {
  if (!n) return PLK_OK;
  const uint64_t b = std::min<uint64_t>((n + 255) / 256, 4096);
  hipLaunchKernelGGL(srs_log_kernel, dim3((unsigned)b), dim3(256), 0, st, d_pts, n, d_logs, d_irregular);
  PLK_HIP(hipGetLastError());
  return PLK_OK;
}

// batch MSMs over log-form points (plk_srs_log_launch); bases and strides 16-byte aligned.
// Blocks per MSM: PLK_OPT_MSM_MAX_BLOCKS (default 2048: one resident round of 256-thread blocks)
// shared by the batch, at most one 16-point group per thread.
int plk_msm_log_batch_launch(const uint8_t* d_logs, uint64_t lstride, const uint8_t* d_sc, uint64_t sstride, uint64_t n,
                             int batch, PlkMsmResult* d_res, hipStream_t st) {
  if (batch <= 0) return PLK_OK;
  if (batch > 65535) {
    plk_set_error("plk_msm batch %d too large", batch);
    return PLK_ERR_RANGE;
  }
  if ((uintptr_t)d_logs % 16 || (uintptr_t)d_sc % 16 || (batch > 1 && (lstride % 16 || sstride % 16))) {
    plk_set_error("plk_msm_log_batch_launch: unaligned operands");
    return PLK_ERR_ARG;
  }
  const uint64_t groups = n >> 4;
  const int64_t env_blocks = plk_opt(PLK_OPT_MSM_MAX_BLOCKS);
  uint64_t b = std::max<uint64_t>(1, (env_blocks > 0 ? (uint64_t)env_blocks : 2048) / (uint64_t)batch);
  b = std::min<uint64_t>(b, std::max<uint64_t>(1, (groups + 255) / 256));
  b = std::min<uint64_t>(b, 8ull * 65535ull);   // the finish's per-shard ticket field is 16 bits
  hipLaunchKernelGGL(msm_log_kernel<256>, dim3((unsigned)b, batch), dim3(256), 0, st, d_logs, lstride, d_sc, sstride, n,
                     d_res);
  PLK_HIP(hipGetLastError());
  return PLK_OK;
}
