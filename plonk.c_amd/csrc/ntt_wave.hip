// Tile-engine NTT passes for transforms of 2^13 .. 2^27 points (poly_mul and plk_ntt_dev).
//
// One block owns one tile of 2^TB elements (TB = 12 or 13): 2^M rows (the pass's butterfly
// bits) x C = 2^(TB-M) columns.  Each thread holds E = 2^R elements in registers: a round
// keeps R consecutive tile bits [lb, lb+R) local to a thread and the other TB-R bits across
// the block's 1024 threads, runs its (<= R) radix-2 stages in registers, and the block
// transposes through a padded LDS buffer between rounds.  The first round loads straight
// from global memory and the last one stores straight back: a pass costs one read + one
// write of the array.  TB, R and M are template parameters, so every round, stage and
// register index is a compile-time constant (no private-memory spills of the register tile).
//
// Plan: the lo = 0 pass takes the low TB bits (contiguous tiles); the bits above are split
// into as few passes as the column width allows (TB = 12: <= 8 bits, >= 16 columns = 64 B
// rows; TB = 13: <= 10 bits, >= 8 columns).  2^13-element tiles (R = 3, 8 elements per
// thread) turn the 3-pass plans of 2^21 .. 2^23 into 2-pass plans: one read + write of the
// array less per transform.
//
// Passes over high bits (lo > 0) need a per-column twiddle w_N^(L * 2^(k-1-s)) at every
// stage s; those factor out of the column transform exactly (checked numerically): a DIF
// pass = plain size-2^M DIF per column, then one multiply of the element at local row r by
// w_{2^(lo+M)}^(L * bitrev_M(r)); a DIT pass = the inverse pre-multiply, then a plain DIT.
// The two table words of each column factor are loaded together with the data, so their
// latency overlaps the tile's load instead of following its last round.
//
// Tiles are placed XCD-aware: blocks b and b+8 share an XCD (observed dispatch, speed
// only), so consecutive tile blocks -- which share cache lines in high-bit passes -- are
// handed to blocks with the same b % 8.
#include "plk_device.h"
#include "plk_internal.h"

#include <stdlib.h>

#include <algorithm>
#include <atomic>
#include <mutex>
#include <type_traits>
#include <vector>

#ifndef PLK_NTT_DIAG
#define PLK_NTT_DIAG 0        // tuning builds only: bit 0 skips the butterflies, bit 1 the LDS exchanges,
                              // bit 2 makes them lane-linear (conflict-free, wrong data), bit 3 loads
                              // one input byte per thread instead of E, bit 4 skips the column-table loads
#endif

namespace {

#ifndef PLK_NTT_R12
#define PLK_NTT_R12 2          // register bits per thread for 2^12 tiles (1024 threads)
#endif
#ifndef PLK_NTT_R13
#define PLK_NTT_R13 3          // ... for 2^13 tiles
#endif
#ifndef PLK_NTT_RC13
#define PLK_NTT_RC13 3         // register bits per thread of the 2^13-tile center kernel
#endif
#ifndef PLK_NTT_BYTE_LUT
#define PLK_NTT_BYTE_LUT 1     // byte values through a 256-entry LDS table (0: arithmetic in registers)
#endif
#ifndef PLK_NTT_SWZ
#define PLK_NTT_SWZ 1          // XOR-swizzled (bank-conflict-free) exchange layout; 0: the 1-in-32 pad
#endif
#ifndef PLK_NTT_CENTER_SWZ
// center exchanges: 3 = the padded layout with barriers only where a wave's element set changes
// (Eng::same_sets; round 5: 2^13 centre 80.2 -> 71.3-72.3 us per launch, prove median 0.394-0.407 ->
// 0.377-0.391 ms, alternating on one box), 0 = padded with a barrier after every exchange's writes
// and reads, 1 / 2 = swizzled everywhere / where the padding conflicts (measured equal to 0)
#define PLK_NTT_CENTER_SWZ 3
#endif
#ifndef PLK_NTT_CENTER_SWZ12
// ... the same for the 2^12-tile center: 4 = one pass-wide conflict-free swizzle with the set-based
// barriers (round 5: poly_mul 2^19 x 2^19 24.14-24.42 -> 23.73-24.07 us alternating; 1 = swizzled
// per exchange, double-buffered, with PLK_NTT_RC12 = 3: 25.2 -> 23.7 us)
#define PLK_NTT_CENTER_SWZ12 4
#endif
#ifndef PLK_NTT_DBUF13
// 2^13-tile high passes: two exchange buffers, one barrier per exchange (round 5: prover forward
// passes 46.8 / 39.2 -> 45.2 / 38.4 us, inverse M = 8 31.1 -> 30.4 us, prove median -0.5..1 %)
#define PLK_NTT_DBUF13 1
#endif
#ifndef PLK_NTT_CENTER_PW
// F29 centres' twiddles as {w, p - w} pairs (no subtraction in the forward DIF): bit 0 = 2^12 tiles
// (round 5: poly_mul 2^19 x 2^19 23.62-23.72 -> 23.34-23.48 us, three alternations), bit 1 = 2^13
// tiles with 2^11 pairs (spills 24-32 B/lane at its 64-VGPR budget: prove median 0.383-0.390 ->
// 0.405-0.417 ms -- off)
#define PLK_NTT_CENTER_PW 1
#endif
#ifndef PLK_NTT_CENTER12_2BUF
#define PLK_NTT_CENTER12_2BUF 0   // the 2^12 centre's b pass in its own buffer (no barrier between a's and b's passes)
#endif
#ifndef PLK_NTT_TRIBUF
#define PLK_NTT_TRIBUF 0       // swizzled double-buffered passes: a third buffer lets wave-local exchanges skip their barrier
#endif
#ifndef PLK_NTT_ALT_ARRAYS
// pass kernels: exchange buffers alternate across a block's arrays, no barrier between arrays (round 5:
// prove median 0.373-0.397 vs 0.377-0.387 ms, four alternations -- off)
#define PLK_NTT_ALT_ARRAYS 0
#endif
#ifndef PLK_NTT_LO_USWZ
// standalone lo = 0 passes: the pass-wide swizzle with set-based barriers (Eng SWZ 4; round 5: 2^20
// forward F29 13.1-13.3 -> 12.5-12.55 us, BabyBear 13.5 -> 12.85-12.9 us, three alternations)
#define PLK_NTT_LO_USWZ 1
#endif
#ifndef PLK_NTT_WRAP_INLINE
#define PLK_NTT_WRAP_INLINE 1  // wrapped tops fixed at the end of the last inverse pass (0: wrap_fix_kernel launches)
#endif
#ifndef PLK_NTT_CW13
#define PLK_NTT_CW13 8         // min waves per SIMD (launch bound): 8 = two 1024-thread blocks per CU
#endif
#ifndef PLK_NTT_CENTER_PF
#define PLK_NTT_CENTER_PF 0    // center: the next item's A loaded during the current item's inverse rounds
#endif
// Round-4 latency-hiding variants, per-kernel times from one box (tools/ab_kernels.sh, prover 2^20,
// forward M = 8 / forward M = 9 / inverse M = 8 passes, us): all off 46.9 / 39.4 / 30.9;
// PREFETCH + XCH_REMAT 45.2 / 38.6 / 31.7 (the inverse passes' prefetch: +0.8, so off there);
// U8_KRSRC alone 50.5 / 43.3 / 30.5 (slower); PREFETCH alone spilled (41.8 us inverse).
#ifndef PLK_NTT_PREFETCH
#define PLK_NTT_PREFETCH 1     // forward pass kernels load array i+1 before array i's butterflies
#endif
#ifndef PLK_NTT_PREFETCH_INV
#define PLK_NTT_PREFETCH_INV 0 // ... and the inverse ones job i+1 before job i's
#endif
#ifndef PLK_NTT_XCH_REMAT
#define PLK_NTT_XCH_REMAT 1    // swizzled exchange addresses recomputed per pass, not held across the array loop
#endif
#ifndef PLK_NTT_M17
#define PLK_NTT_M17 1          // COLT byte outputs: 1 = mod 17 of the index through an LDS table, 0 = 24-bit arithmetic
#endif
#ifndef PLK_NTT_FIX_FILL
#define PLK_NTT_FIX_FILL 0     // the shared-operand lo = 0 launch fills its last round of blocks with operands used once
#endif
#ifndef PLK_NTT_COLI_DERIVE
#define PLK_NTT_COLI_DERIVE 1  // last inverse passes: scaled column factors from the lo / hi roots by products (0: the table)
#endif
#ifndef PLK_NTT_DERIVE
#define PLK_NTT_DERIVE 1       // 2^13-tile first forward passes compute a derived operand (WArrs::derive); 0: compiled out
#endif
#ifndef PLK_NTT_U8_KRSRC
#define PLK_NTT_U8_KRSRC 0     // byte loads: one buffer resource per register index (one offset VGPR)
#endif
#ifndef PLK_NTT_RC12
// register bits per thread of the 2^12-tile center kernel: 3 = 512 threads of 8 elements, 4 rounds of
// 3 stages per transform (3 exchanges instead of 5); with the swizzled exchanges poly_mul 2^19 x 2^19
// 24.95-25.44 -> 23.55-23.85 us (same box, alternating, tools/c3_lib_ab.sh; 2 = 1024 threads)
#define PLK_NTT_RC12 3
#endif
constexpr int wt_rc(int TB) { return TB == 13 ? PLK_NTT_RC13 : PLK_NTT_RC12; }
constexpr int wt_ntc(int TB) { return 1 << (TB - wt_rc(TB)); }
// register bits per thread for a tile size; the block has 2^(TB-R) threads
constexpr int wt_r(int TB) { return TB == 13 ? PLK_NTT_R13 : PLK_NTT_R12; }
constexpr int wt_nt(int TB) { return 1 << (TB - wt_r(TB)); }
constexpr int WT_MAX_HI12 = 8;                 // widest high-bit pass with 2^12 tiles
constexpr int WT_MAX_HI13 = 10;                // ... with 2^13 tiles
constexpr uint32_t M17_LUT = 1040;             // mod-17 table of the byte outputs (F::out17_idx < 1035)

__device__ __forceinline__ int wphys(int e) { return e + (e >> 5); }
// x mod 17 for x < M17_LUT with full-rate 24-bit multiplies: floor(x / 17) = (241 x) >> 12 there
// (checked for every x < 1040), then x - 17 q as one v_mad_i32_i24
__device__ __forceinline__ uint32_t mod17_small(uint32_t x) {
  const uint32_t q = __umul24(x, 241u) >> 12;
  return (uint32_t)(__mul24((int)q, -17) + (int)x);
}

// A tile's words (or bytes) through a buffer resource on its uniform base: every access is one
// 32-bit VGPR offset against scalar registers (no 64-bit address per element; offsets stay below
// 2^30 bytes), and accesses at or past `bytes` are dropped / read 0 -- the byte operands' zero
// padding and the trimmed byte outputs without a per-element branch.
struct TileBuf {
  __amdgpu_buffer_rsrc_t r;
  __device__ __forceinline__ explicit TileBuf(const void* base, uint32_t bytes = 0x7FFFFFF0u)
      : r(__builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, (int)(bytes < 0x7FFFFFF0u ? bytes : 0x7FFFFFF0u),
                                            0x00020000)) {}
  __device__ __forceinline__ uint32_t ld(uint32_t off) const { return __builtin_amdgcn_raw_buffer_load_b32(r, off << 2, 0, 0); }
  __device__ __forceinline__ void st(uint32_t off, uint32_t v) const {
    __builtin_amdgcn_raw_buffer_store_b32(v, r, off << 2, 0, 0);
  }
  // the same with a UNIFORM part of the word offset in the instruction's SGPR offset (no VGPR and
  // no address VALU per register index).  Only for accesses that do not rely on the range check
  // (the words of a tile: the resource's range is unbounded there).
  __device__ __forceinline__ uint32_t ld(uint32_t off, uint32_t uoff) const {
    return __builtin_amdgcn_raw_buffer_load_b32(r, off << 2, uoff << 2, 0);
  }
  __device__ __forceinline__ void st(uint32_t off, uint32_t uoff, uint32_t v) const {
    __builtin_amdgcn_raw_buffer_store_b32(v, r, off << 2, uoff << 2, 0);
  }
  __device__ __forceinline__ uint32_t ldb(uint32_t off) const { return __builtin_amdgcn_raw_buffer_load_b8(r, off, 0, 0); }
  __device__ __forceinline__ void stb(uint32_t off, uint32_t v) const {
    __builtin_amdgcn_raw_buffer_store_b8((uint8_t)v, r, off, 0, 0);
  }
};

struct WPass {
  int k;    // log2 N
  int lo;   // lowest bit of the pass
};

// A batch of independent transforms of one size: job j owns the u32 arrays A (and B for a
// product), optionally reads its inputs as bytes (a8/la, b8/lb) in the first forward pass
// and writes its product as bytes (out8, out_len) in the last inverse pass.
constexpr int WT_MAX_JOBS = PLK_WAVE_MAX_JOBS;
struct WJobs {
  WJob j[WT_MAX_JOBS];
};
// the center launch's item order: slot i holds job[i] (-1: none) for every tile; the grid's
// stride over the items then gives each group of blocks a fixed set of slots (the host balances
// their pass units, center_schedule)
constexpr int WT_SCHED_MAX = 32;
struct WSched {
  int n;    // slots
  int nj;   // jobs of the batch
  int8_t job[WT_SCHED_MAX];
};
// the distinct arrays of a batch that forward passes transform in place (a product's two
// operands, or one standalone transform): u32 array d, first pass from bytes s8[0, ls)
struct WArr {
  uint32_t* d;
  const uint8_t* s8;
  uint64_t ls;
};
constexpr int WT_MAX_ARRS = 2 * WT_MAX_JOBS;
struct WArrs {
  WArr a[WT_MAX_ARRS];
  int derive = 0;   // 1: array 0's bytes are WDerive dv of a[0].s8 (first forward pass only)
  WDerive dv{};
};

struct WTw {
  const uint32_t* small;   // T[2^j + r] = w_{2^(j+1)}^r (Montgomery), 2^PLK_NTT_SMALL_LOG entries
  const uint32_t* lo;      // w_{2^ADIC}^i, i < 4096 (ADIC = the field's 2-adicity)
  const uint32_t* hi;      // w_{2^ADIC}^(4096 i)
  const uint32_t* col;     // forward roots, 2-pass plans: the high pass's column factor of the
                           // element at global index i, fully reduced (nullptr: none)
};

// Field policies.  FBB: BabyBear, values fully reduced in [0, p).  F29: p = 7 2^26 + 1, values
// lazy below 4p (forward) / 8p (inverse) -- bounds in the comments of F29.
//   dif(u, x, w, red)  : u, x <- u + x, (u - x) w;  red = u's inputs may both be >= 2p
//   dit(u, x, w, red)  : u, x <- u + x w, u - x w;  red = u's input may be >= 6p
//   pmul(a, b)         : pointwise product of two forward outputs
//   colf(cl, ch)       : column factor cl * ch, fully reduced (< p)
struct FBB {
  static constexpr int ADIC = bb::TWO_ADICITY;
  __device__ static __forceinline__ void dif(uint32_t& u, uint32_t& x, uint32_t w, bool) {
    const uint32_t a = u, b = x;
    u = bb::madd(a, b);
    x = bb::mmul(bb::msub_lazy(a, b), w);
  }
  __device__ static __forceinline__ void dit(uint32_t& u, uint32_t& x, uint32_t w, bool) {
    const uint32_t xw = bb::mmul(x, w), a = u;
    u = bb::madd(a, xw);
    x = bb::msub(a, xw);
  }
  // stage 0 (twiddle 1): DIF whose outputs go to a column multiply or the stored result; DIT of
  // inputs already < p (what a multiply by one would return)
  __device__ static __forceinline__ void dif1(uint32_t& u, uint32_t& x) {
    const uint32_t a = u, b = x;
    u = bb::madd(a, b);
    x = bb::msub(a, b);   // (reduced: a lo = 0 pass stores it as it is)
  }
  __device__ static __forceinline__ void dit1(uint32_t& u, uint32_t& x, bool) {
    const uint32_t a = u, b = x;
    u = bb::madd(a, b);
    x = bb::msub(a, b);
  }
  __device__ static __forceinline__ void difp(uint32_t& u, uint32_t& x, uint32_t w, uint32_t, bool red) {
    dif(u, x, w, red);
  }
  __device__ static __forceinline__ uint32_t mul(uint32_t a, uint32_t b) { return bb::mmul(a, b); }
  __device__ static __forceinline__ uint32_t pmul(uint32_t a, uint32_t b) { return bb::mmul(a, b); }
  // a + b + c of center outputs (sum groups; c = 0 when absent)
  __device__ static __forceinline__ uint32_t sum(uint32_t a, uint32_t b, uint32_t c) {
    return bb::madd(bb::madd(a, b), c);
  }
  // a + b of two pointwise products, as a pointwise product's bound
  __device__ static __forceinline__ uint32_t add2(uint32_t a, uint32_t b) { return bb::madd(a, b); }
  __device__ static __forceinline__ uint32_t colf(uint32_t cl, uint32_t ch) { return bb::mmul(cl, ch); }
  // a byte's value, NORMAL form (Montgomery twiddles keep a normal-form input normal; the
  // pointwise product's R^-1 is folded into the final scale, see ntt_group)
  __device__ static __forceinline__ uint32_t byte_val(uint32_t b) { return b % 17u; }
  __device__ static __forceinline__ uint32_t out17(uint32_t v, uint32_t ninv) { return bb::mmul(v, ninv) % 17u; }
  // the same when the scale is already applied (the inverse column table holds it)
  __device__ static __forceinline__ uint32_t out17s(uint32_t v) { return v % 17u; }
  // an index < M17_LUT whose entry of the mod-17 table is out17s(v): 2^8 = 1 (mod 17), so a word is
  // congruent to the sum of its bytes (one v_dot4_u32_u8)
  __device__ static __forceinline__ uint32_t out17_idx(uint32_t v) { return __builtin_amdgcn_udot4(v, 0x01010101u, 0u, false); }
  __device__ static __forceinline__ uint32_t scale(uint32_t c, uint32_t ninv) { return bb::mmul(c, ninv); }
  __device__ static __forceinline__ uint32_t canon(uint32_t v) { return v; }   // always reduced
};
// F29 bounds.  Montgomery REDC of t < p 2^32 lands in [0, 2p); so a product of ANY u32 with a
// twiddle w < p is < 2p, and so is the DIF difference term t = a w + b (p - w) (= (a - b) w
// mod p, no subtraction, for any u32 a, b: t <= max(a, b) p).  Forward: every value < 4p;
// x outputs < 2p, so a sum of two x outputs is < 4p as it stands and only a sum of two u
// outputs (< 8p) is reduced (one sub + min); which it is is the element's previous stage bit,
// known at compile time inside a round (the first stage of a round reduces).  Inverse: every
// value < 8p; outputs are a + x w and a + 2p - x w with x w < 2p, so they exceed the a operand's
// bound by 2p and the a operand is reduced (< 8p -> < 4p) when its bound reaches 8p.
struct F29 {
  static constexpr int ADIC = f29::TWO_ADICITY;
  __device__ static __forceinline__ uint32_t red4(uint32_t x) {   // [0, 8p) -> [0, 4p)
    const uint32_t y = x - 2 * f29::P2;
    return y < x ? y : x;
  }
  __device__ static __forceinline__ void dif(uint32_t& u, uint32_t& x, uint32_t w, bool red) {
    const uint32_t a = u, b = x;                 // < 4p
    const uint64_t t = (uint64_t)a * w + (uint64_t)b * (f29::P - w);
    const uint32_t m = (uint32_t)t * f29::PINV;
    x = (uint32_t)((t + (uint64_t)m * f29::P) >> 32);   // < 2p
    const uint32_t s = a + b;                    // < 8p (< 4p when both are x outputs)
    u = red ? red4(s) : s;
  }
  __device__ static __forceinline__ void dit(uint32_t& u, uint32_t& x, uint32_t w, bool red) {
    const uint32_t xw = f29::mmul(x, w);         // any u32 x: [0, 2p)
    const uint32_t a = red ? red4(u) : u;        // a < 6p (unreduced) or < 4p
    u = a + xw;                                  // < a's bound + 2p <= 8p
    x = a + f29::P2 - xw;
  }
  // the same with the twiddle's complement p - w read from the table (no subtraction)
  __device__ static __forceinline__ void difp(uint32_t& u, uint32_t& x, uint32_t w, uint32_t pw, bool red) {
    const uint32_t a = u, b = x;
    const uint64_t t = (uint64_t)a * w + (uint64_t)b * pw;
    const uint32_t m = (uint32_t)t * f29::PINV;
    x = (uint32_t)((t + (uint64_t)m * f29::P) >> 32);
    const uint32_t s = a + b;
    u = red ? red4(s) : s;
  }
  // stage 0 (twiddle 1) of a forward pass whose outputs go to a column multiply (any u32) or to
  // canon ([0, 8p)): a, b < 4p -> both outputs < 8p, no multiply, no reduction
  __device__ static __forceinline__ void dif1(uint32_t& u, uint32_t& x) {
    const uint32_t a = u, b = x;
    u = a + b;
    x = a + 4 * f29::P - b;
  }
  // stage 0 of an inverse pass: its x inputs are < 2p (a pointwise product, a column
  // pre-multiply or canonical data), which is what the multiply by one would have returned
  __device__ static __forceinline__ void dit1(uint32_t& u, uint32_t& x, bool red) {
    const uint32_t xw = x;
    const uint32_t a = red ? red4(u) : u;
    u = a + xw;
    x = a + f29::P2 - xw;
  }
  __device__ static __forceinline__ uint32_t mul(uint32_t a, uint32_t b) { return f29::mmul(a, b); }
  // a + b + c of center outputs (< 8p each): each brought below 2p, the sum < 6p (c = 0 if absent)
  __device__ static __forceinline__ uint32_t sum(uint32_t a, uint32_t b, uint32_t c) {
    return f29::red2(red4(a)) + f29::red2(red4(b)) + f29::red2(red4(c));
  }
  // a, b < 4p: reduce one below 2p so that a b < p 2^32
  __device__ static __forceinline__ uint32_t pmul(uint32_t a, uint32_t b) { return f29::mmul(a, f29::red2(b)); }
  // a + b of two pointwise products (< 2p each), below 2p again (an inverse pass's input bound)
  __device__ static __forceinline__ uint32_t add2(uint32_t a, uint32_t b) { return f29::red2(a + b); }
  __device__ static __forceinline__ uint32_t colf(uint32_t cl, uint32_t ch) { return f29::red1(f29::mmul(cl, ch)); }
  // [0, 8p) -> [0, p): the stored result of a standalone transform
  __device__ static __forceinline__ uint32_t canon(uint32_t v) { return f29::red1(f29::red2(red4(v))); }
  // Centered residues: a coefficient v in [0, 17) enters as v - 17 when v > 8, so every
  // convolution term is at most 64 in absolute value and a product is exact while
  // 64 min(la, lb) <= (p - 1) / 2 (min(la, lb) * 128 < p: up to 3,670,016 coefficients, four
  // times the uncentered bound); a result y > (p - 1) / 2 stands for y - p.
  __device__ static __forceinline__ uint32_t byte_val(uint32_t b) {   // normal form (FBB::byte_val)
    const uint32_t v = b % 17u;
    return v > 8u ? v + (f29::P - 17u) : v;
  }
  __device__ static __forceinline__ uint32_t out17(uint32_t v, uint32_t ninv) {
    const uint32_t y = f29::red1(f29::mmul(v, ninv));
    // y > (p - 1) / 2 stands for y - p = y + C - 17 2^25 with C = 17 2^25 - p > 0: one mod 17
    constexpr uint32_t C = (17u << 25) - f29::P;
    return (y + (y > (f29::P - 1) / 2 ? C : 0u)) % 17u;
  }
  // the same when the scale is already applied (the inverse column table holds it): y < 8p, one
  // reduction to y < 4p; the centered value is c = y - j p with j = floor((y + (p - 1) / 2) / p)
  // (a multiply-high: exact below 6p - 1), and p = 12 mod 17, so c = y + 5 j mod 17
  __device__ static __forceinline__ uint32_t out17s(uint32_t v) {
    const uint32_t y = red4(v);
    const uint32_t j = __umulhi(y + (f29::P - 1) / 2, 2454267022u) >> 28;   // ceil(2^60 / p)
    return (y + 5u * j) % 17u;
  }
  // the same as an index into a mod-17 table (< M17_LUT): y is congruent to the sum of its bytes
  // (2^8 = 1 mod 17), so the centered value is congruent to bytesum(y) + 5 j <= 4 * 255 + 5 * 3
  // (one v_dot4_u32_u8 and a v_mad_u32_u24 instead of the % 17: 3 VALU fewer per output byte)
  __device__ static __forceinline__ uint32_t out17_idx(uint32_t v) {
    const uint32_t y = red4(v);
    const uint32_t j = __umulhi(y + (f29::P - 1) / 2, 2454267022u) >> 28;
    return __builtin_amdgcn_udot4(y, 0x01010101u, 5u * j, false);
  }
  __device__ static __forceinline__ uint32_t scale(uint32_t c, uint32_t ninv) { return f29::red1(f29::mmul(c, ninv)); }
};

// Tile engine: TB tile bits, R local bits per thread (E = 2^R registers, 2^(TB-R) threads
// per tile), a pass of M row bits.  HIGH = the pass is over high index bits (lo > 0):
// exactly the passes with M < TB.  Tiles of 2^12 use double-buffered exchanges (one barrier
// each); 2^13 tiles a single buffer (two barriers) so two blocks fit a CU's LDS.
template <int TB, int R, int M, class F = FBB>
struct Eng {
  static constexpr int E = 1 << R;
  static constexpr int NT = 1 << (TB - R);
  static constexpr bool HIGH = M < TB;
  static constexpr int NR = (M + R - 1) / R;   // rounds
  static constexpr int BUF = (1 << TB) + (1 << TB) / 32;   // padded exchange buffer (words)
  // double-buffered exchanges (one barrier each): 2^12 tiles, and the high passes of 2^13 tiles
  // with PLK_NTT_DBUF13 (2 x 33 KB + their small tables: still two blocks per CU; the lo = 0
  // kernels keep one buffer beside their 2^13-word twiddle table)
  static constexpr bool DBUF = TB <= 12 || (PLK_NTT_DBUF13 && M < TB);
  static constexpr int XCH = NR - 1;            // exchanges per pass
  static constexpr int NBUF = XCH == 0 ? 0 : (XCH > 1 && DBUF ? 2 : 1);

  // DIF rounds take chunks of <= R stage bits from the top (the short chunk last), DIT rounds
  // from the bottom with the short chunk FIRST: either way the first and last rounds of a pass
  // hold R full bits ending at the pass's top or starting at 0, so the column mapping applies
  // to the global loads and stores (a short last DIT round put consecutive threads on
  // different rows: byte stores 2^lo apart, twice the pass time at 2^21).
  static constexpr int s_hi(int q, bool inv) { return inv ? M - 1 - R * (NR - 1 - q) : M - 1 - R * q; }
  static constexpr int s_lo(int q, bool inv) {
    return inv ? (M - R * (NR - q) < 0 ? 0 : M - R * (NR - q))
               : (M - 1 - R * q - (R - 1) < 0 ? 0 : M - 1 - R * q - (R - 1));
  }
  static constexpr int lbq(int q, bool inv) { return s_lo(q, inv) < TB - R ? s_lo(q, inv) : TB - R; }
  // first/last round of a high-bit pass: the low thread bits index the columns, so
  // consecutive threads touch consecutive global addresses.
  static constexpr bool colsq(int q, bool inv) { return HIGH && (q == 0 || q == NR - 1) && lbq(q, inv) + R <= M; }

  // element held by (thread, k) in a round with local bits [lb, lb+R): base(thread) + k << lb
  __device__ static __forceinline__ uint32_t base(uint32_t tid, int lb, bool cols_first) {
    if (!cols_first) return (tid & ((1u << lb) - 1)) | ((tid >> lb) << (lb + R));
    constexpr int cb = TB - M;
    const uint32_t c = tid & ((1u << cb) - 1), rr = tid >> cb;
    return (c << M) | (rr & ((1u << lb) - 1)) | ((rr >> lb) << (lb + R));
  }
  template <int Q>
  __device__ static __forceinline__ uint32_t base_q(uint32_t tid, bool inv) {
    return base(tid, lbq(Q, inv), colsq(Q, inv));
  }

  // the radix-2 stages of round Q, in registers.  Stage 0 has twiddle 1: DIT always skips the
  // multiply there (its x inputs are < 2p, F::dit1), DIF when TRIV0 (a forward pass whose
  // outputs go to the column multiply or the canonical store, F::dif1).  PW: the table holds
  // {w, p - w} pairs (F29 DIF without the subtraction).
  // PWB (the centre's mixed table, PW false): stages s < PWB read {w, p - w} pairs at uint2 index
  // 2^s + r, the others single words at 2^s + r + 2^PWB (0: single words everywhere)
  template <int Q, bool INV, bool PW = false, bool TRIV0 = false, int PWB = 0>
  __device__ static __forceinline__ void round(uint32_t (&v)[E], uint32_t b, const uint32_t* Tsm) {
    if (PLK_NTT_DIAG & 1) return;
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
        // T[2^s + rr] = w_{2^(s+1)}^rr: consecutive rows read consecutive words (no bank
        // conflicts) and the address is linear in the register index, so it folds into the
        // ds_read offset.  (A padded W13 table read at W13[rr << (12 - s)] halved the LDS but
        // needed ~4 VALU of address math per butterfly.)
        // lazy-reduction flags (F29), compile-time after unrolling: DIF reduces u when the
        // pair were u outputs of the previous stage (its bit q+1 of k is 0; unknown for a
        // round's first stage); DIT reduces the a operand on the round's even stages (bound
        // 8p assumed on entry, +2p per stage)
        const bool red = INV ? (i % 2 == 0) : (i == 0 || !((k >> (q + 1)) & 1));
        if (s == 0 && (INV || TRIV0)) {
          if (INV) F::dit1(v[k], v[k | (1 << q)], red);
          else F::dif1(v[k], v[k | (1 << q)]);
          continue;
        }
        if constexpr (PW) {
          const uint2 wp = reinterpret_cast<const uint2*>(Tsm)[(1u << s) + rr];
          F::difp(v[k], v[k | (1 << q)], wp.x, wp.y, red);
          continue;
        }
        if (s < PWB) {   // (compile-time after unrolling)
          const uint2 wp = reinterpret_cast<const uint2*>(Tsm)[(1u << s) + rr];
          if (!INV) F::difp(v[k], v[k | (1 << q)], wp.x, wp.y, red);
          else F::dit(v[k], v[k | (1 << q)], wp.x, red);
          continue;
        }
        const uint32_t w = Tsm[(1u << s) + rr + (PWB ? (1u << PWB) : 0u)];
        if (!INV) F::dif(v[k], v[k | (1 << q)], w, red);
        else F::dit(v[k], v[k | (1 << q)], w, red);
      }
    }
  }

  // ---- exchange layout ------------------------------------------------------------------
  // Tile element bit that thread-id bit i selects in round q's mapping (base() above).
  static constexpr int lane_bit(int q, bool inv, int i) {
    const int lb = lbq(q, inv);
    if (!colsq(q, inv)) return i < lb ? i : i + R;
    if (i < TB - M) return M + i;
    return i - (TB - M) < lb ? i - (TB - M) : i - (TB - M) + R;
  }
  static constexpr bool indep5(const uint32_t* v, int n) {   // linear independence over GF(2)^5
    uint32_t a[8] = {};
    for (int i = 0; i < n; i++) a[i] = v[i];
    int r = 0;
    for (int bit = 0; bit < 5; bit++) {
      int piv = -1;
      for (int i = r; i < n && piv < 0; i++)
        if ((a[i] >> bit) & 1) piv = i;
      if (piv < 0) continue;
      const uint32_t t = a[r];
      a[r] = a[piv];
      a[piv] = t;
      for (int i = 0; i < n; i++)
        if (i != r && ((a[i] >> bit) & 1)) a[i] ^= a[r];
      r++;
    }
    return r == n;
  }
  // Exchange q stores element e at word e ^ h(e), h(e) = XOR of m[j] over the set bits j >= 5 of
  // e (a bijection: only the low 5 bits move).  The bank of a ds_read/ds_write_b32 is (word mod
  // 32) per half-wave, so the 32 lanes are conflict-free iff their 5 varying element bits map to
  // 5 independent bank vectors: unit vectors for element bits < 5, m[j] for the others.  The
  // masks are chosen greedily at compile time so that BOTH the writing round q and the reading
  // round q+1 are conflict-free (checked for every instantiated pass).  With the 1-in-32 pad the
  // column rounds of high passes -- consecutive lanes 2^M words apart -- were 8-way conflicted.
  struct Swz {
    uint32_t m[16];
  };
  static constexpr Swz swz(int q, bool inv) {
    Swz s{};
    int S[2][5] = {};
    for (int i = 0; i < 5; i++) {
      S[0][i] = lane_bit(q, inv, i);
      S[1][i] = lane_bit(q + 1, inv, i);
    }
    for (int j = 5; j < 16; j++) {
      bool in0 = false, in1 = false;
      for (int i = 0; i < 5; i++) {
        in0 = in0 || S[0][i] == j;
        in1 = in1 || S[1][i] == j;
      }
      if (!in0 && !in1) continue;
      for (uint32_t m = 1; m < 32; m++) {
        bool ok = true;
        for (int t = 0; t < 2 && ok; t++) {
          if (!(t ? in1 : in0)) continue;
          uint32_t v[6] = {};
          int n = 0;
          for (int i = 0; i < 5; i++) {
            const int b = S[t][i];
            if (b < 5) v[n++] = 1u << b;
            else if (b < j) v[n++] = s.m[b];
          }
          v[n++] = m;
          ok = indep5(v, n);
        }
        if (ok) {
          s.m[j] = m;
          break;
        }
      }
    }
    return s;
  }
  static constexpr bool swz_ok(int q, bool inv) {   // every lane-bit set got its basis
    const Swz s = swz(q, inv);
    for (int t = 0; t < 2; t++) {
      uint32_t v[5] = {};
      for (int i = 0; i < 5; i++) {
        const int b = lane_bit(q + t, inv, i);
        v[i] = b < 5 ? 1u << b : s.m[b];
      }
      if (!indep5(v, 5)) return false;
    }
    return true;
  }
  // the padded layout (word e + e / 32) is conflict-free for exchange q when the 32 lanes of a
  // half-wave hit 32 distinct banks in both the writing and the reading round
  static constexpr bool pad_ok(int q, bool inv) {
    for (int t = 0; t < 2; t++) {
      bool used[32] = {};
      for (uint32_t l = 0; l < 32; l++) {
        uint32_t e = 0;
        for (int i = 0; i < 5; i++)
          if ((l >> i) & 1) e |= 1u << lane_bit(q + t, inv, i);
        const uint32_t bank = (e + (e >> 5)) & 31u;
        if (used[bank]) return false;
        used[bank] = true;
      }
    }
    return true;
  }
  template <int Q, bool INV>
  __device__ static __forceinline__ uint32_t swz_h(uint32_t e) {
    constexpr Swz s = swz(Q, INV);
    uint32_t h = 0;
#pragma unroll
    for (int j = 5; j < TB; j++)
      if (s.m[j]) h ^= ((e >> j) & 1u) ? s.m[j] : 0u;
    return h;
  }

  // registers (mapping from) -> LDS -> registers (mapping to).  Double-buffered: one barrier
  // suffices (the buffer written next was last read before the previous barrier); single
  // buffer: a second barrier before the buffer is written again.
  // Barriers an exchange needs (round 5).  A round's mapping gives every wave a SET of elements,
  // fixed by the element bits its thread-id bits >= 6 (the wave id) select.  Exchange q writes the
  // wave's round-q set and reads its round-(q + 1) set; with ONE layout for every exchange of a
  // kernel (the padded one, SWZ = 3) two waves' accesses can only meet on a word when their sets
  // differ, so:
  //   * a wave's reads of exchange q and another wave's writes of exchange q + 1 are both of round
  //     q + 1's sets -- disjoint -- so no barrier trails an exchange and one buffer suffices;
  //   * an exchange whose two rounds give every wave the SAME set (wave_local) moves data only
  //     inside each wave, and a wave's LDS operations run in order: no barrier at all;
  //   * between passes (the previous pass's last reads, the next pass's first writes) the caller
  //     puts a barrier unless same_sets says those rounds' sets coincide.
  static constexpr bool same_sets(int qa, bool ia, int qb, bool ib) {
    for (int i = 6; i < TB - R; i++)
      if (lane_bit(qa, ia, i) != lane_bit(qb, ib, i)) return false;
    return true;
  }
  static constexpr bool wave_local(int q, bool inv) { return same_sets(q, inv, q + 1, inv); }
  // One XOR swizzle for EVERY round of a lo = 0 pass in both directions (SWZ = 4): masks m[j] for
  // the element bits j >= 5 that some round puts on a half-wave's 32 lanes, found by depth-first
  // search so that each round's 5 lane vectors are independent (conflict-free); with one layout the
  // barrier rules above hold.  (TB 12 / R 3 and TB 13 / R 3 have one; uswz_ok says so.)
  static constexpr bool uswz_rounds_ok(const uint32_t* m, int upto) {   // rounds whose bits are <= upto
    for (int d = 0; d < 2; d++)
      for (int q = 0; q < NR; q++) {
        uint32_t v[5] = {};
        bool skip = false;
        for (int i = 0; i < 5; i++) {
          const int b = lane_bit(q, d == 1, i);
          if (b > upto) skip = true;
          v[i] = b < 5 ? 1u << b : m[b];
        }
        if (!skip && !indep5(v, 5)) return false;
      }
    return true;
  }
  static constexpr bool uswz_dfs(uint32_t* m, int j) {
    if (j >= TB) return true;
    if (j < 5) return uswz_dfs(m, 5);
    bool used = false;   // does any round put element bit j on a lane?
    for (int d = 0; d < 2; d++)
      for (int q = 0; q < NR; q++)
        for (int i = 0; i < 5; i++) used = used || lane_bit(q, d == 1, i) == j;
    if (!used) {
      m[j] = 0;
      return uswz_dfs(m, j + 1);
    }
    for (uint32_t c = 1; c < 32; c++) {
      m[j] = c;
      if (uswz_rounds_ok(m, j) && uswz_dfs(m, j + 1)) return true;
    }
    m[j] = 0;
    return false;
  }
  static constexpr Swz uswz() {
    Swz s{};
    uswz_dfs(s.m, 5);
    return s;
  }
  static constexpr bool uswz_ok() {
    const Swz s = uswz();
    return uswz_rounds_ok(s.m, 31);
  }
  __device__ static __forceinline__ uint32_t uswz_h(uint32_t e) {
    constexpr Swz s = uswz();
    uint32_t h = 0;
#pragma unroll
    for (int j = 5; j < TB; j++)
      if (s.m[j]) h ^= ((e >> j) & 1u) ? s.m[j] : 0u;
    return h;
  }
  // Three exchange buffers rotating (PLK_NTT_TRIBUF, swizzled double-buffered passes): a wave-local
  // exchange then needs no barrier -- its words are its own wave's, and the block exchanges on
  // either side (the reads of the one before, the writes of the one after, which can run beside it
  // in other waves) use the other two buffers.  Only where no two wave-local exchanges follow each
  // other (longer runs would need more buffers): the 2^12-tile high passes of 7-8 bits.
  static constexpr int wl_run(bool inv) {
    int mx = 0, run = 0;
    for (int q = 0; q + 1 < NR; q++) {
      run = wave_local(q, inv) ? run + 1 : 0;
      mx = run > mx ? run : mx;
    }
    return mx;
  }
  static constexpr bool tri(bool inv) { return PLK_NTT_TRIBUF && DBUF && wl_run(inv) == 1; }
  static constexpr int nbuf() { return XCH == 0 ? 1 : (tri(false) || tri(true) ? 3 : (NBUF ? NBUF : 1)); }
  // the wave's own LDS writes before its reads of other lanes' words (rocPRIM's wave_barrier)
  __device__ static __forceinline__ void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  }

  // SWZ: 0 = the padded layout, 1 = the swizzled layout wherever it is conflict-free, 2 = the
  // swizzled layout only where the padded one conflicts (fewer live address registers: the center),
  // 3 = the padded layout with only the barriers above (one buffer), 4 = the same with the
  // pass-wide swizzle uswz (conflict-free)
  template <int Q, bool INV, int SWZ>
  __device__ static __forceinline__ void exchange(uint32_t (&v)[E], uint32_t* buf, uint32_t bf, int lbf, uint32_t bt,
                                                  int lbt) {
    if (PLK_NTT_DIAG & 2) return;
    if constexpr (SWZ == 4) {
      static_assert(uswz_ok(), "no pass-wide conflict-free swizzle for this tile shape");
      uint32_t xw4 = (bf ^ uswz_h(bf)) << 2, xr4 = (bt ^ uswz_h(bt)) << 2;
      if (PLK_NTT_XCH_REMAT) {
        asm volatile("" : "+v"(xw4));
        asm volatile("" : "+v"(xr4));
      }
      char* bb = reinterpret_cast<char*>(buf);
#pragma unroll
      for (int k = 0; k < E; k++) {
        const uint32_t ek = (uint32_t)k << lbf;
        const uint32_t lo = ((ek & 31u) ^ uswz_h(ek)) << 2, hi = (ek & ~31u) << 2;
        *reinterpret_cast<uint32_t*>(bb + (lo ? (xw4 ^ lo) : xw4) + hi) = v[k];
      }
      if constexpr (wave_local(Q, INV)) wave_sync();
      else __syncthreads();
#pragma unroll
      for (int k = 0; k < E; k++) {
        const uint32_t ek = (uint32_t)k << lbt;
        const uint32_t lo = ((ek & 31u) ^ uswz_h(ek)) << 2, hi = (ek & ~31u) << 2;
        v[k] = *reinterpret_cast<const uint32_t*>(bb + (lo ? (xr4 ^ lo) : xr4) + hi);
      }
      return;
    }
    if constexpr (SWZ == 3) {
#pragma unroll
      for (int k = 0; k < E; k++) buf[wphys((int)(bf + ((uint32_t)k << lbf)))] = v[k];
      if constexpr (wave_local(Q, INV)) wave_sync();
      else __syncthreads();
#pragma unroll
      for (int k = 0; k < E; k++) v[k] = buf[wphys((int)(bt + ((uint32_t)k << lbt)))];
      return;
    }
    if (PLK_NTT_SWZ && SWZ && swz_ok(Q, INV) && (SWZ == 1 || !pad_ok(Q, INV))) {
      // e = base | k << lb (disjoint bits) and h is linear: h(e) = h(base) ^ h(k << lb).  h only
      // moves bits < 5 and the bits >= 5 of k << lb are disjoint from base's, so the word is
      // (xw ^ lo_k) + hi_k: one XOR with a constant (none when lo_k = 0) and the rest in the
      // ds_write / ds_read offset, on byte addresses (no per-element shift)
      uint32_t xw4 = (bf ^ swz_h<Q, INV>(bf)) << 2, xr4 = (bt ^ swz_h<Q, INV>(bt)) << 2;
      if (PLK_NTT_XCH_REMAT) {
        // opaque here: the per-register addresses (xw4 ^ lo) are formed at each use -- one XOR
        // each -- instead of ~7 registers per base live across a kernel's whole array loop
        asm volatile("" : "+v"(xw4));
        asm volatile("" : "+v"(xr4));
      }
      char* bb = reinterpret_cast<char*>(buf);
#pragma unroll
      for (int k = 0; k < E; k++) {
        const uint32_t ek = (uint32_t)k << lbf;
        const uint32_t lo = ((ek & 31u) ^ swz_h<Q, INV>(ek)) << 2, hi = (ek & ~31u) << 2;
        *reinterpret_cast<uint32_t*>(bb + (lo ? (xw4 ^ lo) : xw4) + hi) = v[k];
      }
      if constexpr (tri(INV) && wave_local(Q, INV)) wave_sync();
      else __syncthreads();
#pragma unroll
      for (int k = 0; k < E; k++) {
        const uint32_t ek = (uint32_t)k << lbt;
        const uint32_t lo = ((ek & 31u) ^ swz_h<Q, INV>(ek)) << 2, hi = (ek & ~31u) << 2;
        v[k] = *reinterpret_cast<const uint32_t*>(bb + (lo ? (xr4 ^ lo) : xr4) + hi);
      }
      if (!DBUF) __syncthreads();
      return;
    }
    if (PLK_NTT_DIAG & 4) {   // timing only: conflict-free lane-linear exchange (wrong data)
#pragma unroll
      for (int k = 0; k < E; k++) buf[k * NT + threadIdx.x] = v[k];
      __syncthreads();
#pragma unroll
      for (int k = 0; k < E; k++) v[k] = buf[k * NT + (threadIdx.x ^ 1)];
      if (!DBUF) __syncthreads();
      return;
    }
#pragma unroll
    for (int k = 0; k < E; k++) buf[wphys((int)(bf + ((uint32_t)k << lbf)))] = v[k];
    if constexpr (tri(INV) && wave_local(Q, INV) && SWZ < 3) wave_sync();
    else __syncthreads();
#pragma unroll
    for (int k = 0; k < E; k++) v[k] = buf[wphys((int)(bt + ((uint32_t)k << lbt)))];
    if (!DBUF) __syncthreads();
  }

  // rounds Q .. NR-1 of a pass; registers hold the mapping of round Q on entry and of the
  // last round on exit.  xc selects the exchange buffer (it counts exchanges).
  // SWZ: the swizzled exchange layout where it is conflict-free (the center kernel passes false:
  // it has no VGPRs to spare for the two extra base registers)
  template <bool INV, int SWZ = 1, bool PW = false, bool TRIV0 = false, int PWB = 0, int Q = 0>
  __device__ static __forceinline__ void pass(uint32_t (&v)[E], uint32_t tid, uint32_t* bufs, int xc,
                                              const uint32_t* Tsm) {
    round<Q, INV, PW, TRIV0, PWB>(v, base_q<Q>(tid, INV), Tsm);
    if constexpr (Q + 1 < NR) {
      exchange<Q, INV, SWZ>(v, bufs + (!DBUF || SWZ >= 3 ? 0 : (tri(INV) ? ((xc + Q) % 3) : ((xc + Q) & 1)) * BUF),
                            base_q<Q>(tid, INV), lbq(Q, INV),
                            base_q<Q + 1>(tid, INV), lbq(Q + 1, INV));
      pass<INV, SWZ, PW, TRIV0, PWB, Q + 1>(v, tid, bufs, xc, Tsm);
    }
  }

  // global index of tile-local element e = c * 2^M + r
  __device__ static __forceinline__ uint64_t index(const WPass& p, uint32_t tile, uint32_t e) {
    if (M == TB) return ((uint64_t)tile << TB) | e;
    constexpr int cb = TB - M;
    const uint32_t r = e & ((1u << M) - 1), c = e >> M;
    const int sh = p.lo - cb;                          // tiles per H row = 2^sh
    const uint64_t H = tile >> sh;
    const uint32_t L = ((tile & ((1u << sh) - 1)) << cb) | c;
    return (H << (p.lo + M)) | ((uint64_t)r << p.lo) | L;
  }

  // the same index split into a uniform tile base and a 32-bit offset (no shared bits):
  // index = tbase + toff(e), toff < 2^(lo + M) <= 2^k
  __device__ static __forceinline__ uint64_t tbase(const WPass& p, uint32_t tile) {
    if (M == TB) return (uint64_t)tile << TB;
    constexpr int cb = TB - M;
    const int sh = p.lo - cb;
    return ((uint64_t)(tile >> sh) << (p.lo + M)) | ((uint64_t)(tile & ((1u << sh) - 1)) << cb);
  }
  __device__ static __forceinline__ uint32_t toff(const WPass& p, uint32_t e) {
    if (M == TB) return e;
    return ((e & ((1u << M) - 1)) << p.lo) | (e >> M);
  }
  // offset of element b + (k << lb) of round q: the register index k only moves row bits when
  // lb + R <= M (every column-mapped round), so it is toff(b) + (k << (lb + lo))
  template <int Q, bool INV>
  __device__ static __forceinline__ uint32_t toff_k(const WPass& p, uint32_t o0, uint32_t b, int k) {
    constexpr int LB = lbq(Q, INV);
    if constexpr (M == TB || LB + R <= M) return o0 + (((uint32_t)k << LB) << (M == TB ? 0 : p.lo));   // (lo = 0 when M = TB)
    else return toff(p, b + ((uint32_t)k << LB));
  }

  // toff_k as (per-lane o0, UNIFORM per-k part) when the register index only moves row bits --
  // every column-mapped round and the lo = 0 pass: word access k of the thread = o0 + kpart(k)
  template <int Q, bool INV>
  static constexpr bool ksplit() { return M == TB || lbq(Q, INV) + R <= M; }
  template <int Q, bool INV>
  __device__ static __forceinline__ uint32_t kpart(const WPass& p, int k) {
    return ((uint32_t)k << lbq(Q, INV)) << (M == TB ? 0 : p.lo);
  }
  // a tile's word k of round Q's mapping through a TileBuf: the split form where it applies
  template <int Q, bool INV>
  __device__ static __forceinline__ uint32_t ldk(const TileBuf& t, const WPass& p, uint32_t o0, uint32_t b, int k) {
    if constexpr (ksplit<Q, INV>()) return t.ld(o0, kpart<Q, INV>(p, k));
    else return t.ld(toff_k<Q, INV>(p, o0, b, k));
  }
  template <int Q, bool INV>
  __device__ static __forceinline__ void stk(const TileBuf& t, const WPass& p, uint32_t o0, uint32_t b, int k, uint32_t v) {
    if constexpr (ksplit<Q, INV>()) t.st(o0, kpart<Q, INV>(p, k), v);
    else t.st(toff_k<Q, INV>(p, o0, b, k), v);
  }

  // column factor exponent (in w_{2^27} units) for element e of a high-bit pass
  __device__ static __forceinline__ uint32_t col_exp(const WPass& p, uint32_t tile, uint32_t e) {
    constexpr int cb = TB - M;
    const uint32_t r = e & ((1u << M) - 1), c = e >> M;
    const int sh = p.lo - cb;
    const uint32_t L = ((tile & ((1u << sh) - 1)) << cb) | c;
    const uint32_t f = __brev(r) >> (32 - M);
    return (L * f) << (F::ADIC - p.lo - M);   // w_{2^(lo+M)}^(L f) in w_{2^ADIC} units
  }
};

// tile of this block, XCD-aware: consecutive tiles go to blocks with equal b % 8
__device__ __forceinline__ uint32_t block_tile() {
  const uint32_t nb = gridDim.x, b = blockIdx.x;
  return (nb % 8 == 0) ? (b % 8) * (nb / 8) + b / 8 : b;
}

// the pass's stage twiddles into LDS: the first 2^M entries of the table T
template <int M, int NT>
__device__ __forceinline__ void load_pass_tw(uint32_t* Tsm, const uint32_t* small) {
  const TileBuf bs(small);   // (32-bit offsets: nothing 64-bit for the compiler to hoist and spill)
#pragma unroll
  for (int i = 0; i < ((1 << M) + NT - 1) / NT; i++) {
    const int j = i * NT + (int)threadIdx.x;
    if (j < (1 << M)) Tsm[j] = bs.ld((uint32_t)j);
  }
}

// the centre's mixed table (Eng::round's PWB): {w, p - w} pairs for the first 2^PWB entries, the
// others as single words at their index + 2^PWB (2^TB + 2^PWB words)
template <int TB, int PWB, int NT>
__device__ __forceinline__ void load_center_tw(uint32_t* T, const uint32_t* small) {
  const TileBuf bs(small);
#pragma unroll
  for (int i = 0; i < ((1 << TB) + NT - 1) / NT; i++) {
    const int j = i * NT + (int)threadIdx.x;
    if (j < (1 << TB)) {
      const uint32_t w = bs.ld((uint32_t)j);
      if (j < (1 << PWB)) reinterpret_cast<uint2*>(T)[j] = make_uint2(w, f29::P - w);
      else T[j + (1 << PWB)] = w;
    }
  }
}

// the same as {w, p - w} pairs (F29 forward passes)
template <int M, int NT>
__device__ __forceinline__ void load_pass_tw_pairs(uint32_t* Tsm, const uint32_t* small) {
#pragma unroll
  for (int i = 0; i < ((1 << M) + NT - 1) / NT; i++) {
    const int j = i * NT + (int)threadIdx.x;
    if (j < (1 << M)) {
      const uint32_t w = TileBuf(small).ld((uint32_t)j);
      reinterpret_cast<uint2*>(Tsm)[j] = make_uint2(w, f29::P - w);
    }
  }
}

// Array 0 of a derived batch (WArrs::derive): the bytes of round 3's A2 B2 at the elements this
// thread loads (WDerive; the same map as prove.hip's t2a_kernel, exact mod 17), also stored to the
// operand's bytes ar.s8 [0, ar.ls).  Byte offsets are element indices (< 2^27); a[i - 1] at i = 0
// is the offset 2^32 - 1, out of every range: 0.
template <class G>
__device__ __forceinline__ void load_derived(const WArrs& arrs, WPass p, uint64_t tb, uint32_t o0, uint32_t b0,
                                             uint32_t (&v)[G::E]) {
  const WDerive& dv = arrs.dv;
  const WArr& ar = arrs.a[0];
  const uint32_t al = dv.S[dv.s_alpha], be = dv.S[dv.s_beta], ga = dv.S[dv.s_gamma], bk1 = dv.S[dv.s_bk1];
  const TileBuf bab(dv.ab, (uint32_t)(dv.lab < 0x7FFFFFF0ull ? dv.lab : 0x7FFFFFF0ull));
  const TileBuf ba(dv.a, (uint32_t)(dv.la < 0x7FFFFFF0ull ? dv.la : 0x7FFFFFF0ull));
  const TileBuf bb(dv.b, (uint32_t)(dv.la < 0x7FFFFFF0ull ? dv.la : 0x7FFFFFF0ull));
  const TileBuf bo(ar.s8, (uint32_t)(ar.ls < 0x7FFFFFF0ull ? ar.ls : 0x7FFFFFF0ull));
  uint32_t ix[G::E], wab[G::E], ak[G::E], bk[G::E], am[G::E], bm[G::E];
#pragma unroll
  for (int k = 0; k < G::E; k++) {
    ix[k] = (uint32_t)tb + G::template toff_k<0, false>(p, o0, b0, k);
    wab[k] = bab.ldb(ix[k]);
    ak[k] = ba.ldb(ix[k]);
    bk[k] = bb.ldb(ix[k]);
    am[k] = ba.ldb(ix[k] - 1u);
    bm[k] = bb.ldb(ix[k] - 1u);
  }
#pragma unroll
  for (int k = 0; k < G::E; k++) {
    const uint32_t i = ix[k];
    // (gamma + beta x)(gamma + beta k1 x) at x^0, x^1, x^2
    const uint32_t K = i == 0 ? ga * ga : i == 1 ? ga * (bk1 + be) : i == 2 ? be * bk1 : 0u;
    // (bound: 16 + 16 * 32 + 2 * 16 * 16 + 289 < 2^11)
    const uint32_t x = wab[k] + ga * (ak[k] + bk[k]) + bk1 * am[k] + be * bm[k] + K;
    v[k] = (x % 17u) * al % 17u;
    bo.stb(i, v[k]);
  }
}

}  // namespace

// Forward (DIF) pass over a batch's distinct arrays, u32 in place, or the first pass reading
// bytes (zero padded, reduced mod 17, to Montgomery).  Block (x, y) runs tile x of arrays
// y apa .. y apa + apa - 1 (< na) one after another: the arrays' column factors at a tile are the
// same words, so they are loaded once per block (and the stage twiddles too).
// COLT: the column factors come from tw.col (one word per element, indexed like the data)
// instead of lo * hi (two words and a multiply per element).
template <int TB, int R, int M, bool FROM_U8, class F, bool COLT = false>
__global__ __launch_bounds__(wt_nt(TB), TB == 13 && M == TB ? 4 : 8) void wt_fwd_kernel(WPass p, WArrs arrs, WTw tw, int na,
                                                                                       int apa) {
  using G = Eng<TB, R, M, F>;
  static_assert(G::NT == wt_nt(TB), "tile block size");
  constexpr bool PW = F::ADIC == f29::TWO_ADICITY;   // {w, p - w} pairs (F29's lazy DIF)
  __shared__ __attribute__((aligned(16))) uint32_t Tsm[(PW ? 2 : 1) << M];
  __shared__ uint32_t bufs[G::nbuf() * G::BUF];
  const uint32_t tid = threadIdx.x;
  const uint32_t tile = block_tile();

  // uniform tile base pointers, 32-bit element offsets
  const uint64_t tb = G::tbase(p, tile);
  const uint32_t* colt = COLT ? tw.col + tb : nullptr;
  const uint32_t b0 = G::template base_q<0>(tid, false);
  const uint32_t o0 = G::toff(p, b0);
  // this thread's elements of array ai: raw bytes (0 past the operand: the buffer's range ends
  // there; their values through an LDS table after the barrier) or words
  auto load = [&](int ai, uint32_t (&v)[G::E]) {
    const WArr& ar = arrs.a[ai];
    if constexpr (FROM_U8) {
      const uint64_t ls = ar.ls;
      const uint32_t lim = ls > tb ? (uint32_t)(ls - tb < 0xFFFFFFFFull ? ls - tb : 0xFFFFFFFFull) : 0u;
      if constexpr (PLK_NTT_U8_KRSRC && !(PLK_NTT_DIAG & 8) && G::template ksplit<0, false>()) {
        // register index k reads byte o0 + kpart(k): its own resource based at kpart(k) with the
        // range shortened by as much, so one offset VGPR serves all E loads and the range check
        // still zero-pads past the operand
#pragma unroll
        for (int k = 0; k < G::E; k++) {
          const uint32_t kp = G::template kpart<0, false>(p, k);
          v[k] = TileBuf(ar.s8 + tb + kp, lim > kp ? lim - kp : 0u).ldb(o0);
          if (!PLK_NTT_BYTE_LUT) v[k] = F::byte_val(v[k]);
        }
        return;
      }
      const TileBuf bs(ar.s8 + tb, lim);
#pragma unroll
      for (int k = 0; k < G::E; k++) {
        const uint32_t o = G::template toff_k<0, false>(p, o0, b0, k);
        if ((PLK_NTT_DIAG & 8) && k > 0) { v[k] = (v[0] + k) & 0xFFu; continue; }
        v[k] = bs.ldb(o);
        if (!PLK_NTT_BYTE_LUT) v[k] = F::byte_val(v[k]);
      }
    } else {
      const TileBuf bd(ar.d + tb);
#pragma unroll
      for (int k = 0; k < G::E; k++) v[k] = G::template ldk<0, false>(bd, p, o0, b0, k);
    }
  };
  int ai = (int)blockIdx.y * apa;
  uint32_t v[G::E];
  // (the first array's loads go out before the tables'; a derived array is array 0, so only a
  // block's first load can be one -- never a prefetch)
  // (2^13 tiles only: the 2^12-tile byte passes -- C3's poly_mul -- keep their registers, 36 VGPRs
  // instead of 40: poly_mul 2^19 x 2^19 +0.3 us with the branch compiled in)
  if (PLK_NTT_DERIVE && TB == 13 && FROM_U8 && ai == 0 && arrs.derive) load_derived<G>(arrs, p, tb, o0, b0, v);
  else load(ai, v);
  // column factor table words of the elements this thread stores (HIGH passes): the same for
  // every array of the block
  constexpr int LF = G::lbq(G::NR - 1, false);
  const uint32_t bf = G::template base_q<G::NR - 1>(tid, false);
  const uint32_t of = G::toff(p, bf);
  uint32_t cl[G::HIGH ? G::E : 1], ch[G::HIGH && !COLT ? G::E : 1];
  if (G::HIGH) {
#pragma unroll
    for (int k = 0; k < G::E; k++) {
      if constexpr (COLT) {
        cl[k] = (PLK_NTT_DIAG & 16) ? 0x12345u + k : G::template ldk<G::NR - 1, false>(TileBuf(colt), p, of, bf, k);
      } else {
        const uint32_t ex = G::col_exp(p, tile, bf + ((uint32_t)k << LF));
        cl[k] = tw.lo[ex & 4095u];
        ch[k] = tw.hi[ex >> 12];
      }
    }
  }
  __shared__ uint32_t lut[FROM_U8 && PLK_NTT_BYTE_LUT ? 256 : 1];
  if (FROM_U8 && PLK_NTT_BYTE_LUT && tid < 256) lut[tid] = F::byte_val(tid);
  if constexpr (PW) load_pass_tw_pairs<M, G::NT>(Tsm, tw.small);
  else load_pass_tw<M, G::NT>(Tsm, tw.small);
  // exchange layout: the lo = 0 pass of a standalone transform may take the pass-wide swizzle
  constexpr int XSWZ = M == TB && PLK_NTT_LO_USWZ ? 4 : 1;
  // (xc continues over the arrays: with alternating buffers the one an array's first exchange
  // writes was last read before the previous array's last exchange barrier -- no barrier needed)
  constexpr bool ALT = PLK_NTT_ALT_ARRAYS && G::DBUF && XSWZ < 3;
  for (int q = 0;; q++) {
    // (q = 0: the tables are in LDS; q > 0 without ALT: every thread's reads of the previous
    // array's last exchange are done before this one's first exchange writes)
    if (q == 0 || !ALT) __syncthreads();
    if constexpr (FROM_U8 && PLK_NTT_BYTE_LUT) {
#pragma unroll
      for (int k = 0; k < G::E; k++) v[k] = lut[v[k]];
    }
    const bool more = q + 1 < apa && ai + 1 < na;   // (uniform)
    // the next array's loads go out before this one's rounds, so their latency hides behind the
    // butterflies (the barriers wait for LDS only: the loads stay in flight across them)
    uint32_t nv[G::E];
    if (PLK_NTT_PREFETCH && more) load(ai + 1, nv);
    G::template pass<false, XSWZ, PW, true>(v, tid, bufs, ALT ? q * G::XCH : 0, Tsm);
    const TileBuf bd(arrs.a[ai].d + tb);
#pragma unroll
    for (int k = 0; k < G::E; k++) {
      uint32_t x = v[k];
      if constexpr (G::HIGH && COLT) x = F::mul(x, cl[k]);
      else if constexpr (G::HIGH) x = F::mul(x, F::colf(cl[k], ch[k]));
      else x = F::canon(x);   // the lo = 0 pass is the last one of a standalone transform
      G::template stk<G::NR - 1, false>(bd, p, of, bf, k, x);
    }
    if (!more) break;
    ++ai;
    if constexpr (PLK_NTT_PREFETCH) {
#pragma unroll
      for (int k = 0; k < G::E; k++) v[k] = nv[k];
    } else {
      load(ai, v);
    }
  }
}


// Wrapped products (la + lb - 1 = N + ntop): the last inverse pass wrote c[j] + c[N + j] mod 17
// at j < ntop.  c[N + j] (sum group: of the group's sum) has only the terms a[i] b[N + j - i]
// with i > N + j - lb (ntop - j <= 16 of them): computed from the bytes after the pass, by this
// small launch (round 4: inlined into the pass kernel, its loops held registers in the hot path).
// Block = job (jobs without a wrapped top return at once), thread j < ntop = position j; a job
// with a trimmed-length word takes the positions' maximum into it (the pass left them out).
// Every term a[i] b[N + j - i] of c[N + j] (j < ntop <= 16) has i in the top 16 bytes of a and
// N + j - i in the top 16 of b (la + lb - 1 - N <= 16, also for a group's shorter members): the
// block stages those bytes in LDS with ONE load each, then thread j sums from LDS -- one memory
// round trip for the whole fix (a loop of dependent byte loads per term took ~5 us per launch).
__global__ __launch_bounds__(64) void wrap_fix_kernel(WJobs jobs, uint64_t N) {
  const WJob& jb = jobs.j[blockIdx.x];
  const uint32_t ntop = (uint32_t)jb.ntop;
  if (!ntop) return;   // (uniform: a job without a wrapped top)
  __shared__ uint32_t A[3][16], B[3][16];   // [member][q] = byte la - 16 + q (0 below index 0)
  const uint32_t t = threadIdx.x;
  if (t < 48) {
    const int g = (int)(t >> 4), q = (int)(t & 15);
    uint32_t va = 0, vb = 0;
    if (g <= jb.ngroup) {
      const uint8_t* a = g ? jb.ga8[g - 1] : jb.a8;
      const uint8_t* b = g ? jb.gb8[g - 1] : jb.b8;
      const uint64_t la = g ? jb.gla[g - 1] : jb.la, lb = g ? jb.glb[g - 1] : jb.lb;
      if (la + (uint64_t)q >= 16) va = a[la - 16 + q] % 17u;
      if (lb + (uint64_t)q >= 16) vb = b[lb - 16 + q] % 17u;
    }
    A[g][q] = va;
    B[g][q] = vb;
  }
  const uint32_t j = t;
  const uint32_t cur = j < ntop ? jb.out8[j] : 0u;   // (c[j] + c[N + j] mod 17, the pass's byte)
  __syncthreads();
  if (j >= ntop) return;
  uint32_t s = 0;
  for (int g = 0; g <= jb.ngroup; g++) {
    const uint64_t la = g ? jb.gla[g - 1] : jb.la, lb = g ? jb.glb[g - 1] : jb.lb;
    if (la + lb - 1 <= N + j) continue;   // (a shorter member: no term reaches c[N + j])
    // i in [N + j + 1 - lb, la): q = i - la + 16, b index N + j - i = lb - 16 + (16 + N + j + lb... )
    const int d = (int)(la + lb - 1 - N - j);   // terms: i = la - d .. la - 1 (d <= 16)
#pragma unroll
    for (int u = 0; u < 16; u++) {
      // i = la - d + u: a at q = 16 - d + u, b index N + j - i = lb - 1 - u: q = 15 - u
      if (u < d) s += A[g][16 - d + u] * B[g][15 - u];
    }
  }
  s %= 17u;
  const uint32_t lo = (cur + 17u - s) % 17u;
  jb.out8[j] = (uint8_t)lo;
  jb.out8[N + j] = (uint8_t)s;
  uint32_t last = lo ? j + 1u : 0u;
  if (s) last = (uint32_t)(N + j) + 1u;
  if (jb.nz && last) atomicMax(jb.nz, last);
}

// Inverse (DIT) pass, u32 in place (the job's C); the final pass (TO_U8) scales by N^-1 (normal form,
// which also leaves Montgomery form), reduces mod 17 and writes bytes for idx < out_len.
// COLT (final passes only): the column table is the inverse one, whose factors carry that scale
// (the pass is linear), so the bytes come from the pass's outputs directly (F::out17s).
// Block (x, y) runs tile x of jobs y jpb .. y jpb + jpb - 1 (< nj) one after another, loading the
// column factors and stage twiddles once for all of them.
template <int TB, int R, int M, bool TO_U8, class F, bool COLT = false>
__global__ __launch_bounds__(wt_nt(TB), 8) void wt_inv_kernel(WPass p, WJobs jobs, WTw tw, uint32_t ninv, int nj, int jpb) {
  using G = Eng<TB, R, M, F>;
  static_assert(G::NT == wt_nt(TB), "tile block size");
  // prefetch where the registers allow it: the wide byte-output passes have none to spare (their
  // spill reloads would wait for the prefetched loads anyway)
  constexpr bool PF = PLK_NTT_PREFETCH_INV && !(TO_U8 && (M > 8 || M < 4));
  __shared__ uint32_t Tsm[1 << M];
  __shared__ uint32_t bufs[G::nbuf() * G::BUF];
  const uint32_t tid = threadIdx.x;
  const uint32_t tile = block_tile();

  // uniform tile base pointers, 32-bit element offsets
  const uint64_t tb = G::tbase(p, tile);
  const uint32_t* colt = COLT ? tw.col + tb : nullptr;
  const uint32_t b0 = G::template base_q<0>(tid, true);
  const uint32_t o0 = G::toff(p, b0);
  constexpr int L0 = G::lbq(0, true);
  int ji = (int)blockIdx.y * jpb;
  uint32_t v[G::E];
  auto load = [&](int j, uint32_t (&x)[G::E]) {
    const TileBuf bd(jobs.j[j].C + tb);
#pragma unroll
    for (int k = 0; k < G::E; k++) x[k] = G::template ldk<0, true>(bd, p, o0, b0, k);
  };
  load(ji, v);   // (the first job's loads go out before the tables')
  uint32_t cl[G::HIGH ? G::E : 1], ch[G::HIGH && !COLT ? G::E : 1];
  if constexpr (G::HIGH && COLT && PLK_NTT_COLI_DERIVE && G::colsq(0, true)) {
    // The scaled column factors without the table (the 2^22 table is 16 MiB read per
    // launch).  Round 0 is column-mapped: a thread's E words share their column L and differ only in
    // the row bits [L0, L0 + R), so their exponents are ex0 + sum over the set register bits b of d_b
    // (bitrev of disjoint bits adds).  cl[0] = scale(w^ex0) from the lo / hi roots, d_b's roots the
    // same way, then each cl[k] = cl[k - 2^b] * w^(d_b) for k's top bit b: R + 1 root lookups and
    // E - 1 + R + 2 multiplies per thread for all of the block's jobs.  Every product is fully
    // reduced, so the words equal the table's (tests: the prover goldens, poly_mul vs the oracle).
    // (Passes narrower than a round, M < R + L0, keep the table: their registers leave the row.)
    const uint32_t e0 = G::col_exp(p, tile, b0);
    cl[0] = F::scale(F::colf(tw.lo[e0 & 4095u], tw.hi[e0 >> 12]), ninv);
#pragma unroll
    for (int b = 0; (1 << b) < G::E; b++) {
      const uint32_t d = G::col_exp(p, tile, b0 + (1u << (L0 + b))) - e0;
      const uint32_t g = F::colf(tw.lo[d & 4095u], tw.hi[d >> 12]);
#pragma unroll
      for (int k = 1 << b; k < (2 << b) && k < G::E; k++) cl[k] = F::colf(cl[k - (1 << b)], g);
    }
  } else if (G::HIGH) {
#pragma unroll
    for (int k = 0; k < G::E; k++) {
      if constexpr (COLT) {
        cl[k] = G::template ldk<0, true>(TileBuf(colt), p, o0, b0, k);
      } else {
        const uint32_t ex = G::col_exp(p, tile, b0 + ((uint32_t)k << L0));   // roots of tw (inverse or forward)
        cl[k] = tw.lo[ex & 4095u];
        ch[k] = tw.hi[ex >> 12];
      }
    }
  }
  load_pass_tw<M, G::NT>(Tsm, tw.small);
  // (COLT byte outputs) x mod 17 for x < M17_LUT, read at F::out17_idx
  __shared__ uint8_t m17[TO_U8 && COLT && PLK_NTT_M17 ? M17_LUT : 1];
  if constexpr (TO_U8 && COLT && PLK_NTT_M17) {
    for (uint32_t i = tid; i < M17_LUT; i += G::NT) m17[i] = (uint8_t)(i % 17u);
  }
  const uint32_t bf = G::template base_q<G::NR - 1>(tid, true);
  const uint32_t of = G::toff(p, bf);
  const uint32_t N = 1u << p.k;   // (k <= 27: every index fits 32 bits)
  constexpr int XSWZ = M == TB && PLK_NTT_LO_USWZ ? 4 : 1;
  constexpr bool ALT = PLK_NTT_ALT_ARRAYS && G::DBUF && XSWZ < 3;
  for (int q = 0;; q++) {
    const WJob& jb = jobs.j[ji];   // (sum-group members are not in the grid: no inverse of their own)
    uint8_t* out8 = jb.out8;
    const uint64_t out_len = jb.out_len;
    const uint32_t* s1 = jb.S1;
    const uint32_t* s2 = jb.S2;
    if (s1) {   // a sum group's leader (uniform): its members' center outputs, all loads in flight
      const uint32_t* s1t = s1 + tb;
      const uint32_t* s2t = s2 ? s2 + tb : nullptr;
      uint32_t a1[G::E], a2[G::E];
#pragma unroll
      for (int k = 0; k < G::E; k++) {
        a1[k] = G::template ldk<0, true>(TileBuf(s1t), p, o0, b0, k);
        a2[k] = s2 ? G::template ldk<0, true>(TileBuf(s2t), p, o0, b0, k) : 0u;
      }
#pragma unroll
      for (int k = 0; k < G::E; k++) v[k] = F::sum(v[k], a1[k], a2[k]);
    }
    if (G::HIGH) {
#pragma unroll
      for (int k = 0; k < G::E; k++) {
        if constexpr (COLT) v[k] = F::mul(v[k], cl[k]);
        else v[k] = F::mul(v[k], F::colf(cl[k], ch[k]));
      }
    }
    const bool more = q + 1 < jpb && ji + 1 < nj;   // (uniform)
    // the next job's loads before this one's rounds (wt_fwd_kernel)
    uint32_t nv[G::E];
    if (PF && more) load(ji + 1, nv);
    // (q = 0: the stage twiddles are in LDS; q > 0 without ALT: the previous job's last exchange
    // reads are done; with ALT the buffers alternate over the jobs, wt_fwd_kernel)
    if (q == 0 || !ALT) __syncthreads();
    G::template pass<true, XSWZ>(v, tid, bufs, ALT ? q * G::XCH : 0, Tsm);
    uint32_t last = 0;      // 1 + the largest index this thread left a non-zero byte at
    const uint32_t lim = out_len < N ? (uint32_t)out_len : N;
    const uint32_t ntop = (uint32_t)jb.ntop;   // (read once: the byte stores below may alias the job table)
    if constexpr (!TO_U8) {
      const TileBuf bd(jb.C + tb);
#pragma unroll
      for (int k = 0; k < G::E; k++)   // (the standalone inverse's last pass; poly_mul's 3-pass middle one)
        G::template stk<G::NR - 1, true>(bd, p, of, bf, k, F::canon(v[k]));
    } else {
      // poly_mul runs its inverse with the FORWARD roots (no inverse table in LDS): that yields
      // N c[-idx mod N], so the coefficient lands at the negated position.  Every byte is computed
      // before the first store (the stores then issue back to back).
      // (the buffer's range is the output length: bytes at or past it are dropped by the store)
      const TileBuf bo(out8, lim);
      uint32_t jj[G::E], rr[G::E];
#pragma unroll
      for (int k = 0; k < G::E; k++) {
        jj[k] = (N - ((uint32_t)tb + G::template toff_k<G::NR - 1, true>(p, of, bf, k))) & (N - 1);
        rr[k] = !COLT ? F::out17(v[k], ninv)
                : PLK_NTT_M17 ? (uint32_t)m17[F::out17_idx(v[k])] : mod17_small(F::out17_idx(v[k]));
      }
#pragma unroll
      for (int k = 0; k < G::E; k++) bo.stb(jj[k], rr[k]);
      // the trimmed length only when the job has one (uniform: the prover's batched products do
      // not; the wrapped positions j < ntop are fixed, and counted, by wrap_fix_kernel)
      if (jb.nz) {
#pragma unroll
        for (int k = 0; k < G::E; k++) last = max(last, (jj[k] < lim && jj[k] >= ntop && rr[k]) ? jj[k] + 1u : 0u);
      }
    }

    // Trimmed length (src/poly.h:20-38).  The top coefficient of a single product is
    // a[la-1] b[lb-1] mod 17 (one term, wrapped or not); when it is non-zero -- operands with
    // non-zero leading bytes, the usual case -- the length is la + lb - 1 and one store says so.
    // Otherwise every tile takes its block's maximum into the word (zeroed by the center kernel).
    if (TO_U8 && jb.nz) {
      const bool top = jb.ngroup == 0 && (jb.a8[jb.la - 1] % 17u) * (jb.b8[jb.lb - 1] % 17u) % 17u != 0u;
      if (top) {
        if (blockIdx.x == 0 && tid == 0) *jb.nz = (uint32_t)(out_len + (uint64_t)jb.ntop);
      } else {
        last = plk_block_max(last);
        if (tid == 0 && last) atomicMax(jb.nz, last);
      }
    }
    if (!more) break;
    ++ji;
    if constexpr (PF) {
#pragma unroll
      for (int k = 0; k < G::E; k++) v[k] = nv[k];
    } else {
      load(ji, v);
    }
  }
#if PLK_NTT_WRAP_INLINE
  // Wrapped tops (wrap_fix_kernel's work, done by the block whose tile holds the position, after
  // its jobs: no launch of its own).  Position j < ntop is element (N - j) mod N.
  if constexpr (TO_U8) {
    const int j0 = (int)blockIdx.y * jpb;
    bool any = false;
    for (int q = j0; q <= ji; q++) any |= jobs.j[q].ntop > 0;
    if (any) {
      __builtin_amdgcn_s_waitcnt(0);   // this thread's byte stores complete ...
      __syncthreads();                 // ... and every other thread's
      for (int q = j0; q <= ji; q++) {
        const WJob& jb = jobs.j[q];
        const uint32_t ntop = (uint32_t)jb.ntop, j = tid;
        if (j >= ntop) continue;
        const uint32_t idx = (N - j) & (N - 1);
        uint32_t tl;   // the tile of element idx (Eng::index inverted)
        if (M == TB) {
          tl = idx >> TB;
        } else {
          constexpr int cb = TB - M;
          const int sh = p.lo - cb;
          tl = ((idx >> (p.lo + M)) << sh) | ((idx & ((1u << p.lo) - 1)) >> cb);
        }
        if (tl != tile) continue;
        uint32_t sum = 0;
        for (int g = 0; g <= jb.ngroup; g++) {
          const uint8_t* a = g ? jb.ga8[g - 1] : jb.a8;
          const uint8_t* b = g ? jb.gb8[g - 1] : jb.b8;
          const uint64_t la = g ? jb.gla[g - 1] : jb.la, lb = g ? jb.glb[g - 1] : jb.lb;
          if (la + lb - 1 <= (uint64_t)N + j) continue;
          const int d = (int)(la + lb - 1 - N - j);   // terms i = la - d + u, b index lb - 1 - u
          uint32_t av[16], bv[16];
#pragma unroll
          for (int u = 0; u < 16; u++) {
            av[u] = u < d ? a[la - d + u] : 0u;
            bv[u] = u < d ? b[lb - 1 - u] : 0u;
          }
#pragma unroll
          for (int u = 0; u < 16; u++) sum += (av[u] % 17u) * (bv[u] % 17u);
        }
        const uint32_t sv = sum % 17u;
        const uint32_t lo = (jb.out8[j] + 17u - sv) % 17u;
        jb.out8[j] = (uint8_t)lo;
        jb.out8[N + j] = (uint8_t)sv;
        uint32_t lst = lo ? j + 1u : 0u;
        if (sv) lst = N + j + 1u;
        if (jb.nz && lst) atomicMax(jb.nz, lst);
      }
    }
  }
#endif
}

// Center of poly_mul: last forward pass (lo = 0) of a and b, pointwise product (plus a merged
// sum group's member products), first inverse pass, all in registers of one block; result
// written to the job's C (A, B or a free array: A and B may be read by other jobs of the batch).  The last DIF round
// and the first DIT round both have local bits [0, R), so no exchange sits in between.
// Stage twiddles: ONE table T in LDS (2^TB words): the inverse runs with the forward roots
// (the DIT of the forward DFT; the final pass negates output positions, wt_inv_kernel), which
// halves the block's LDS so that two blocks fit a CU.
// GRP: the launch has merged sum groups (the item loop's per-pair steps; without, one pair)
template <int TB, int R, class F, bool GRP>
__global__ __launch_bounds__(wt_ntc(TB), TB == 13 ? PLK_NTT_CW13 : 1) void wt_center_kernel(WPass p, WJobs jobs,
                                                                                                     WTw twf, WSched sc) {
  using G = Eng<TB, R, TB, F>;
  static_assert(G::NT == wt_ntc(TB), "tile block size");
  static_assert(G::lbq(G::NR - 1, false) == 0 && G::lbq(0, true) == 0, "center mapping");
  constexpr int CSWZ = TB == 13 ? PLK_NTT_CENTER_SWZ : PLK_NTT_CENTER_SWZ12;
  constexpr bool UNI = CSWZ >= 3;   // one layout, barriers only where sets change (Eng::same_sets)
  // (UNI, 2^12 tiles, PLK_NTT_CENTER12_2BUF) b's pass in a buffer of its own: a's last reads and b's
  // first writes cannot meet, so no barrier between the two forward passes (the inverse pass, back in
  // a's buffer, starts after b's first barrier, when every wave has left a's pass)
  constexpr bool B2 = UNI && TB == 12 && PLK_NTT_CENTER12_2BUF;
  static_assert(!B2 || !G::wave_local(0, false), "b's first exchange must carry the barrier that ends a's pass");
  // (F29, PLK_NTT_CENTER_PW) the twiddle table's low stages as {w, p - w} pairs: the forward DIF
  // skips its p - w subtraction there; 2^11 pairs for 2^13 tiles keep two blocks per CU in LDS
  constexpr int CPWB = F::ADIC != f29::TWO_ADICITY ? 0
                       : TB == 13 ? ((PLK_NTT_CENTER_PW & 2) ? 11 : 0) : ((PLK_NTT_CENTER_PW & 1) ? TB : 0);
  __shared__ __attribute__((aligned(16))) uint32_t Tlds[(1 << TB) + (CPWB ? (1 << CPWB) : 0)];
  __shared__ uint32_t bufs[(G::DBUF && (!UNI || B2) ? 2 : 1) * G::BUF];
  const uint32_t* Tf = Tlds;
  const uint32_t tid = threadIdx.x;
  const uint32_t b0 = G::template base_q<0>(tid, false);
  constexpr int L0 = G::lbq(0, false);
  constexpr int LF = G::lbq(G::NR - 1, true);
  const uint32_t bf = G::template base_q<G::NR - 1>(tid, true);
  // persistent: the grid (<= 2 blocks per CU) walks the batch's (slot, tile) items, so the
  // 2^TB-word twiddle table is loaded once per block instead of once per tile
  const uint32_t tiles = (uint32_t)((1ull << p.k) >> TB), items = tiles * (uint32_t)sc.n;
  // trimmed-length words of the jobs that want one: zeroed here, before the last inverse pass
  if (blockIdx.x == 0 && tid < (uint32_t)sc.nj && jobs.j[tid].nz) *jobs.j[tid].nz = 0u;
  // the twiddle table first (a "first item" flag inside the loop had the compiler hoist the
  // table's addresses out of the loop and spill them)
  if constexpr (CPWB) load_center_tw<TB, CPWB, G::NT>(Tlds, twf.small);
  else load_pass_tw<TB, G::NT>(Tlds, twf.small);
  // the item after `it` in this block's stride that has a job (items of padding slots skipped)
  auto next_item = [&](uint32_t it) {
    for (it += gridDim.x; it < items && sc.job[it / tiles] < 0; it += gridDim.x) {
    }
    return it;
  };
  uint32_t pa[G::E];   // (PLK_NTT_CENTER_PF) the next item's A words, loaded during this item's inverse rounds
  bool have = false;   // (uniform) pa holds this item's A
  for (uint32_t it = blockIdx.x; it < items; it += gridDim.x) {
    const uint32_t slot = it / tiles, tile = it - slot * tiles;
    const int job = sc.job[slot];
    if (job < 0) continue;   // (uniform: a padding slot)
    const WJob& J = jobs.j[job];
    // (the lo = 0 pass: a tile is 2^TB consecutive words; 32-bit offsets from its base)
    const uint64_t tb = (uint64_t)tile << TB;
    const TileBuf b_c(J.C + tb);
    uint32_t va[G::E], vb[G::E];
    int xc = 0;
    // the job's pair, then a merged sum group's members' pairs: each pointwise product but the
    // last is parked in the job's C tile (its own positions; C is no operand of the group) and
    // added to the next one, so two register arrays suffice
    for (int q = 0;; q++) {
      const WJob& P = jobs.j[q ? J.cm[q - 1] : job];
      const TileBuf b_a(P.A + tb), b_b(P.B + tb);
      // (a block's first item loads its A here; later ones found it prefetched)
      const bool pre = PLK_NTT_CENTER_PF && q == 0 && have;
#pragma unroll
      for (int k = 0; k < G::E; k++) {
        va[k] = pre ? pa[k] : b_a.ld(b0, (uint32_t)k << L0);   // (the per-register part in the SGPR offset)
        vb[k] = b_b.ld(b0, (uint32_t)k << L0);
      }
      // (the previous item's or pair's last exchange reads; with UNI the previous pair's too.
      // Skipping it where Eng::same_sets allows -- the inverse's last round and the forward's first
      // give the waves the same sets -- measured no faster: kept)
      if (q == 0 || UNI) __syncthreads();
      // (afix / bfix: the operand's transform is finished -- plk_wave_pretransform / wt_fixfwd_kernel
      // stored this pass's output registers where their inputs were read -- so its pass is
      // skipped; xc counts the exchanges so that double buffers keep alternating)
      if (!P.afix) {
        G::template pass<false, CSWZ, false, false, CPWB>(va, tid, bufs, xc, Tf);
        xc += G::XCH;
      }
      if (!P.bfix) {
        // (UNI: a's last reads against b's first writes)
        if (UNI && !B2 && !P.afix && !G::same_sets(G::NR - 1, false, 0, false)) __syncthreads();
        G::template pass<false, CSWZ, false, false, CPWB>(vb, tid, B2 ? bufs + G::BUF : bufs, xc, Tf);
        xc += G::XCH;
      }
#pragma unroll
      for (int k = 0; k < G::E; k++) va[k] = F::pmul(va[k], vb[k]);
      if (GRP && q) {
#pragma unroll
        for (int k = 0; k < G::E; k++) va[k] = F::add2(va[k], b_c.ld(b0, (uint32_t)k << L0));
      }
      if (!GRP || q == J.ncm) break;
#pragma unroll
      for (int k = 0; k < G::E; k++) b_c.st(b0, (uint32_t)k << L0, va[k]);
      __builtin_amdgcn_s_waitcnt(0);   // (the parked words are this thread's own: stored before reloaded)
    }
    if (PLK_NTT_CENTER_PF) {
      // the next item's A goes out before this one's inverse rounds (no job writes an array
      // another job reads, and the same job's next item is another tile)
      const uint32_t nit = next_item(it);
      have = nit < items;
      if (have) {
        const uint32_t ns = nit / tiles;
        const TileBuf b_n(jobs.j[sc.job[ns]].A + ((uint64_t)(nit - ns * tiles) << TB));
#pragma unroll
        for (int k = 0; k < G::E; k++) pa[k] = b_n.ld(b0, (uint32_t)k << L0);
      }
    }
    // (UNI: the forward passes' last reads against the inverse pass's first writes)
    if (UNI && !G::same_sets(G::NR - 1, false, 0, true)) __syncthreads();
    G::template pass<true, CSWZ, false, false, CPWB>(va, tid, bufs, xc, Tf);
#pragma unroll
    for (int k = 0; k < G::E; k++) b_c.st(bf, (uint32_t)k << LF, va[k]);
  }
}

// The lo = 0 forward pass of a fixed operand, exactly as wt_center_kernel runs it on b, each
// thread storing its output registers where it read its inputs (so a later center launch loads
// them unchanged: WJob::bfix / afix).  In place: every position is read and written by one
// thread.  blockIdx.y = which array.
template <int TB, int R, class F>
__global__ __launch_bounds__(wt_ntc(TB), TB == 13 ? PLK_NTT_CW13 : 1) void wt_fixfwd_kernel(WPass p, WArrs arrs,
                                                                                                    WTw twf) {
  using G = Eng<TB, R, TB, F>;
  constexpr int CSWZ0 = TB == 13 ? PLK_NTT_CENTER_SWZ : PLK_NTT_CENTER_SWZ12;
  constexpr int CSWZ = CSWZ0 >= 3 ? CSWZ0 : 0;
  uint32_t* d = arrs.a[blockIdx.y].d;
  __shared__ uint32_t Tlds[1 << TB];
  __shared__ uint32_t bufs[(G::DBUF && CSWZ < 3 ? 2 : 1) * G::BUF];
  const uint32_t tid = threadIdx.x, tile = blockIdx.x;
  const uint32_t b0 = G::template base_q<0>(tid, false);
  constexpr int L0 = G::lbq(0, false);
  uint32_t v[G::E];
  const TileBuf bt(d + ((uint64_t)tile << TB));   // (the lo = 0 pass: consecutive words)
#pragma unroll
  for (int k = 0; k < G::E; k++) v[k] = bt.ld(b0, (uint32_t)k << L0);
  load_pass_tw<TB, G::NT>(Tlds, twf.small);
  __syncthreads();
  G::template pass<false, CSWZ>(v, tid, bufs, G::XCH, Tlds);
#pragma unroll
  for (int k = 0; k < G::E; k++) bt.st(b0, (uint32_t)k << L0, v[k]);
}

// Column-factor table of a 2-pass plan (lo = TB, M = k - TB): entry i = the high pass's factor
// of the element at global index i = r 2^lo + L, w_{2^k}^(L bitrev_M(r)), fully reduced; with
// ninv != 0 the product's final scale times that factor (the table of the last inverse pass).
template <int TB, class F>
__global__ __launch_bounds__(256) void coltab_kernel(uint32_t* __restrict__ out, int k, WTw tw, uint32_t ninv) {
  const uint64_t idx = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  if (idx >= (1ull << k)) return;
  const int M = k - TB;
  const uint32_t L = (uint32_t)(idx & ((1u << TB) - 1)), r = (uint32_t)(idx >> TB);
  const uint32_t f = M ? __brev(r) >> (32 - M) : 0u;
  const uint32_t ex = (L * f) << (F::ADIC - k);
  const uint32_t c = F::colf(tw.lo[ex & 4095u], tw.hi[ex >> 12]);
  out[idx] = ninv ? F::scale(c, ninv) : c;
}

// ------------------------------------------------------------------------------ host side
namespace {

// tile bits for a 2^k transform: 2^13 tiles from PLK_OPT_NTT_T13_MIN_K (default 21) up
int tile_bits(int k) { return k >= plk_opt(PLK_OPT_NTT_T13_MIN_K) ? 13 : 12; }

// resident blocks of the persistent center kernel: 2 per CU (PLK_OPT_NTT_CENTER_BLOCKS overrides)
uint32_t center_blocks() {
  static std::atomic<uint32_t> resident{0};
  if (const int64_t o = plk_opt(PLK_OPT_NTT_CENTER_BLOCKS)) return (uint32_t)o;
  uint32_t nb = resident.load(std::memory_order_relaxed);
  if (!nb) {
    int dev = 0, cus = 256;
    if (hipGetDevice(&dev) == hipSuccess) (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    // the resident blocks: the launch bound's waves per SIMD x 4 SIMDs over the block's waves
    const uint32_t per_cu = std::max<uint32_t>(1u, (uint32_t)PLK_NTT_CW13 * 4u * 64u / (uint32_t)wt_ntc(13));
    nb = per_cu * (uint32_t)(cus > 0 ? cus : 256);
    resident.store(nb, std::memory_order_relaxed);
  }
  return nb;
}

// passes of a 2^k transform, high bits first: the bits above the TB-bit lo = 0 pass in
// balanced chunks of <= 8 (TB 12) / 10 (TB 13) bits
int wave_plan(int k, int TB, int* Ms) {
  const int hi = k - TB, mx = TB == 12 ? WT_MAX_HI12 : WT_MAX_HI13;
  const int nh = (hi + mx - 1) / mx;
  int n = 0;
  for (int i = 0; i < nh; i++) Ms[n++] = hi / nh + (i < hi % nh ? 1 : 0);
  Ms[n++] = TB;
  return n;
}

// a 2^k transform's plan has one high pass (the column tables' case, coltab_kernel)
bool two_pass(int k) { return k - tile_bits(k) <= (tile_bits(k) == 12 ? WT_MAX_HI12 : WT_MAX_HI13); }

// column tables [field][k] (field 0 BabyBear, 1 F29) for the 2-pass plans, k = 13 .. 23
#ifndef PLK_NTT_COLT_MIN_K
#define PLK_NTT_COLT_MIN_K 13   // smallest transform using a column table (tuning: larger = lo * hi products)
#endif
constexpr int COLT_MIN_K = 13, COLT_MAX_K = 23;
// per device (plk_cur_device: the calling thread's current device)
uint32_t* g_col[PLK_MAX_DEVICES][2][COLT_MAX_K + 1] = {};
uint32_t* g_coli[PLK_MAX_DEVICES][2][COLT_MAX_K + 1] = {};   // the same times the product's final scale (ntt.hip's ninv)

WTw to_wtw(const PlkTwTables& t, bool inv) {
  return inv ? WTw{t.small_i, t.lo_i, t.hi_i, nullptr} : WTw{t.small_f, t.lo_f, t.hi_f, nullptr};
}
// forward roots of field F with the column table of a 2^k transform (when built)
template <class F>
WTw fwd_wtw(int k) {
  const bool f29 = F::ADIC == f29::TWO_ADICITY;
  WTw w = to_wtw(f29 ? plk_ntt_tables29() : plk_ntt_tables(), false);
  // (a table holds the factors of the plan's ONE high pass: a three-pass plan's top pass -- 2^12
  // tiles above 2^20 when PLK_OPT_NTT_T13_MIN_K moves the 2^13 threshold up -- multiplies lo * hi)
  w.col = (k >= PLK_NTT_COLT_MIN_K && k >= COLT_MIN_K && k <= COLT_MAX_K && two_pass(k))
              ? g_col[plk_cur_device()][f29 ? 1 : 0][k]
              : nullptr;
  return w;
}
// the same for a product's last inverse pass: the scaled column table
template <class F>
WTw inv_wtw(int k) {
  WTw w = fwd_wtw<F>(k);
  if (w.col) w.col = g_coli[plk_cur_device()][F::ADIC == f29::TWO_ADICITY ? 1 : 0][k];
  return w;
}

// the table path applies to the pass whose bits reach the top (lo + M = k): a plan's first
// forward and last inverse pass; byte-input forward / byte-output inverse or single-array
// forward passes are the only ones instantiated with it
// Diagnostics (PLK_OPT_NTT_LAUNCH_LOG = 1): the launch plans of the tile engine's passes, in launch
// order, for the offline roofline tools (tools/ntt_roofline.py, tools/ntt_pmc_summary.py --plan):
// a profiler records a launch's grid, not how many arrays its blocks walk (per_block below) or
// how many pass units the persistent center kernel runs.  kind: 0 forward pass, 1 inverse pass,
// 2 center (n = products, units = lo = 0 passes run per tile), 3 shared-operand lo = 0 pass;
// field 0 = F29, 1 = BabyBear (bench.py prices each launch against its field's butterfly peak).
struct LaunchRec {
  int32_t kind, tb, m, k, n, per_block, units, field;
};
std::mutex g_log_mu;
std::vector<LaunchRec> g_log;
template <class F>
void log_launch(int kind, int tb, int m, int k, int n, int per_block, int units) {
  if (!plk_opt(PLK_OPT_NTT_LAUNCH_LOG)) return;
  std::lock_guard<std::mutex> lk(g_log_mu);
  if (g_log.size() < 65536)
    g_log.push_back(LaunchRec{kind, tb, m, k, n, per_block, units, std::is_same<F, F29>::value ? 0 : 1});
}

// Arrays (jobs) per block of a table pass: several arrays of one tile share its column-table words
// (read once per block instead of once per array: the 2^22 table is 16 MiB); chosen so that the
// launch's rounds of resident blocks (2 per CU) times the arrays per block stay at their minimum
// (one array per block: ceil(tiles n / resident)), the largest such count.
// PLK_OPT_NTT_TABLE_SHARE = 0: one array per block.
int per_block(uint32_t tiles, int n) {
  if (!plk_opt(PLK_OPT_NTT_TABLE_SHARE) || n <= 1) return 1;
  static std::atomic<int> cus{0};
  int c = cus.load(std::memory_order_relaxed);
  if (!c) {
    int dev = 0;
    c = 256;
    if (hipGetDevice(&dev) == hipSuccess) (void)hipDeviceGetAttribute(&c, hipDeviceAttributeMultiprocessorCount, dev);
    if (c <= 0) c = 256;
    cus.store(c, std::memory_order_relaxed);
  }
  const uint64_t res = 2ull * (uint64_t)c;   // resident 1024-thread blocks: 2 per CU
  auto cost = [&](int J) { return ((tiles * (uint64_t)((n + J - 1) / J) + res - 1) / res) * (uint64_t)J; };
  int best = 1;
  for (int J = 2; J <= n; J++)
    if (cost(J) <= cost(best)) best = J;
  return best;
}

template <int TB, int M, bool U8, class F>
void launch_fwd(WPass p, const WArrs& arrs, int na, WTw tw, hipStream_t st) {
  constexpr int R = wt_r(TB);
  const uint32_t tiles = (uint32_t)((1ull << p.k) >> TB);
  if constexpr (M < TB) {
    if (tw.col && p.lo + M == p.k) {
      const int J = per_block(tiles, na);
      log_launch<F>(0, TB, M, p.k, na, J, 0);
      hipLaunchKernelGGL((wt_fwd_kernel<TB, R, M, U8, F, true>), dim3(tiles, (na + J - 1) / J), dim3(wt_nt(TB)), 0, st, p,
                         arrs, tw, na, J);
      return;
    }
  }
  log_launch<F>(0, TB, M, p.k, na, 1, 0);
  hipLaunchKernelGGL((wt_fwd_kernel<TB, R, M, U8, F>), dim3(tiles, na), dim3(wt_nt(TB)), 0, st, p, arrs, tw, na, 1);
}
template <int TB, int M, bool U8, class F>
void launch_inv(WPass p, const WJobs& jobs, int nj, WTw tw, uint32_t ninv, hipStream_t st) {
  constexpr int R = wt_r(TB);
  const uint32_t tiles = (uint32_t)((1ull << p.k) >> TB);
  if constexpr (M < TB && U8) {
    if (tw.col && p.lo + M == p.k) {
      const int J = per_block(tiles, nj);
      log_launch<F>(1, TB, M, p.k, nj, J, 0);
      hipLaunchKernelGGL((wt_inv_kernel<TB, R, M, U8, F, true>), dim3(tiles, (nj + J - 1) / J), dim3(wt_nt(TB)), 0, st, p,
                         jobs, tw, ninv, nj, J);
      return;
    }
  }
  log_launch<F>(1, TB, M, p.k, nj, 1, 0);
  hipLaunchKernelGGL((wt_inv_kernel<TB, R, M, U8, F>), dim3(tiles, nj), dim3(wt_nt(TB)), 0, st, p, jobs, tw, ninv, nj, 1);
}

// pass widths: 1..8 for both tile sizes, 9..10 for 2^13 tiles, M = TB for the lo = 0 pass
template <int TB, bool U8, class F>
int fwd_m(int M, WPass p, const WArrs& arrs, int na, WTw tw, hipStream_t st) {
#define PLK_FWD(m) launch_fwd<TB, m, U8, F>(p, arrs, na, tw, st)
  switch (M) {
    case 1: PLK_FWD(1); break;
    case 2: PLK_FWD(2); break;
    case 3: PLK_FWD(3); break;
    case 4: PLK_FWD(4); break;
    case 5: PLK_FWD(5); break;
    case 6: PLK_FWD(6); break;
    case 7: PLK_FWD(7); break;
    case 8: PLK_FWD(8); break;
    default:
      if constexpr (TB == 13) {
        if (M == 9) { PLK_FWD(9); break; }
        if (M == 10) { PLK_FWD(10); break; }
      }
      if constexpr (!U8) {
        if (M == TB) { launch_fwd<TB, TB, false, F>(p, arrs, na, tw, st); break; }
      }
      plk_set_error("wave plan: unsupported pass width %d (tile bits %d)", M, TB);
      return PLK_ERR_ARG;
  }
#undef PLK_FWD
  PLK_HIP(hipGetLastError());
  return PLK_OK;
}

template <int TB, bool U8, class F>
int inv_m(int M, WPass p, const WJobs& jobs, int nj, WTw tw, uint32_t ninv, hipStream_t st) {
#define PLK_INV(m) launch_inv<TB, m, U8, F>(p, jobs, nj, tw, ninv, st)
  switch (M) {
    case 1: PLK_INV(1); break;
    case 2: PLK_INV(2); break;
    case 3: PLK_INV(3); break;
    case 4: PLK_INV(4); break;
    case 5: PLK_INV(5); break;
    case 6: PLK_INV(6); break;
    case 7: PLK_INV(7); break;
    case 8: PLK_INV(8); break;
    default:
      if constexpr (TB == 13) {
        if (M == 9) { PLK_INV(9); break; }
        if (M == 10) { PLK_INV(10); break; }
      }
      if constexpr (!U8) {
        if (M == TB) { launch_inv<TB, TB, false, F>(p, jobs, nj, tw, ninv, st); break; }
      }
      plk_set_error("wave plan: unsupported pass width %d (tile bits %d)", M, TB);
      return PLK_ERR_ARG;
  }
#undef PLK_INV
  PLK_HIP(hipGetLastError());
  return PLK_OK;
}

// pass units of a center job's item (the lo = 0 passes it runs; 0: no item)
int center_units(const WJobs& cj, int j) {
  const WJob& J = cj.j[j];
  if (J.cskip) return 0;
  int u = !J.afix + !J.bfix + 1;
  for (int q = 0; q < J.ncm; q++) u += !cj.j[J.cm[q]].afix + !cj.j[J.cm[q]].bfix;
  return u;
}

// The center launch's item order.  The grid strides over (slot, tile) items, so with tiles
// dividing the grid, blocks [b T, (b + 1) T) take exactly the slots b, b + bins, b + 2 bins, ...
// (bins = grid / T): the jobs go to bins by decreasing pass units, each to the bin with the
// fewest so far (padding slots where the bins' job counts differ).  Otherwise the job order.
WSched center_schedule(const WJobs& cj, int nj, uint32_t T, uint32_t nb) {
  WSched s{};
  s.nj = nj;
  int list[WT_MAX_JOBS], units[WT_MAX_JOBS], n = 0;
  for (int j = 0; j < nj; j++)
    if ((units[j] = center_units(cj, j)) > 0) list[n++] = j;
  const uint64_t G = std::min<uint64_t>((uint64_t)T * n, nb);
  const uint32_t bins = G % T == 0 ? (uint32_t)(G / T) : 0u;
  if (bins > 1 && (uint64_t)T * n > G) {
    std::stable_sort(list, list + n, [&](int a, int b) { return units[a] > units[b]; });
    int bl[WT_SCHED_MAX][WT_MAX_JOBS], cnt[WT_SCHED_MAX] = {}, load[WT_SCHED_MAX] = {}, mx = 0;
    bool ok = bins <= WT_SCHED_MAX;
    for (int i = 0; i < n && ok; i++) {
      uint32_t b = 0;
      for (uint32_t c = 1; c < bins; c++)
        if (load[c] < load[b]) b = c;
      bl[b][cnt[b]++] = list[i];
      load[b] += units[list[i]];
      mx = std::max(mx, cnt[b]);
    }
    if (ok && bins * (uint32_t)mx <= WT_SCHED_MAX) {
      s.n = (int)bins * mx;
      for (int i = 0; i < s.n; i++) {
        const uint32_t b = (uint32_t)i % bins, r = (uint32_t)i / bins;
        s.job[i] = (int8_t)((int)r < cnt[b] ? bl[b][r] : -1);
      }
      return s;
    }
  }
  s.n = n;
  for (int i = 0; i < n; i++) s.job[i] = (int8_t)list[i];
  return s;
}

// Sum groups: the leader's center item adds its members' pointwise products (members without
// items, the leader's inverse pass without their center outputs)
void merge_groups(WJobs& cj, WJobs& ij, int nj) {
  for (int L = 0; L < nj; L++) {
    if (!ij.j[L].S1) continue;
    int mem[2], nm = 0;
    for (int j = 0; j < nj; j++)
      if (j != L && (cj.j[j].C == ij.j[L].S1 || (ij.j[L].S2 && cj.j[j].C == ij.j[L].S2)) && nm < 2) mem[nm++] = j;
    if (nm != (ij.j[L].S2 ? 2 : 1)) continue;
    for (int q = 0; q < nm; q++) {
      cj.j[L].cm[q] = mem[q];
      cj.j[mem[q]].cskip = 1;
    }
    cj.j[L].ncm = nm;
    ij.j[L].S1 = ij.j[L].S2 = nullptr;
  }
}

template <int TB, class F>
int wave_poly_mul_t(const WJobs& jobs, int nj, int k, uint32_t ninv, hipStream_t st) {
  PLK_MARK(4);
  const WTw twf = fwd_wtw<F>(k);   // forward roots for the inverse too (wt_center_kernel)
  int Ms[4];
  const int np = wave_plan(k, TB, Ms);
  int lo[4];
  for (int i = 0, top = k; i < np; i++) { lo[i] = top - Ms[i]; top = lo[i]; }
  // the distinct operand arrays (jobs may share one)
  WArrs arrs{};
  int na = 0;
  for (int j = 0; j < nj; j++)
    for (int s = 0; s < (jobs.j[j].bfix ? 1 : 2); s++) {   // (a finished b has no forward passes)
      const WArr a = s ? WArr{jobs.j[j].B, jobs.j[j].b8, jobs.j[j].lb} : WArr{jobs.j[j].A, jobs.j[j].a8, jobs.j[j].la};
      bool seen = false;
      for (int q = 0; q < na; q++) seen |= arrs.a[q].d == a.d;
      if (!seen) arrs.a[na++] = a;
    }
  // a derived operand (PlkPolyMulJob::der) becomes array 0: the first forward pass computes it
  for (int j = 0; j < nj; j++) {
    if (!jobs.j[j].der) continue;
    int q = 0;
    while (q < na && arrs.a[q].d != jobs.j[j].A) q++;
    if (!PLK_NTT_DERIVE || TB != 13 || arrs.derive || np < 2 || q == na || jobs.j[j].der->la < 1) {
      plk_set_error("wave poly_mul: a derived operand needs 2^13 tiles, one per batch and two or more passes "
                    "(2^%d: %d-bit tiles, %d passes)", k, TB, np);
      return PLK_ERR_ARG;
    }
    std::swap(arrs.a[0], arrs.a[q]);
    arrs.derive = 1;
    arrs.dv = *jobs.j[j].der;
  }
  int rc;
  PLK_MARK(5);
  for (int i = 0; i < np - 1; i++) {
    const WPass p{k, lo[i]};
    rc = i == 0 ? fwd_m<TB, true, F>(Ms[i], p, arrs, na, twf, st) : fwd_m<TB, false, F>(Ms[i], p, arrs, na, twf, st);
    if (rc) return rc;
  }
  PLK_MARK(6);
  const uint32_t tiles = (uint32_t)((1ull << k) >> TB);
  // operands shared by several products of the batch: their lo = 0 forward pass runs once, in
  // its own launch, instead of once per product inside the center items (PLK_OPT_NTT_SHARED_FIX
  // 0: off, 2: also next to pretransformed operands).  The extra launch moves a tile's loads and
  // stores besides its pass (768 tiles: 18.6 us against 20 us less center time in the prover's
  // 2^21 batch): within the ~10 us run-to-run spread of a proof's kernel span either way
  // (tools/prove_ab_prof.sh, medians over 4-5 calls), so batches holding a pretransformed
  // operand keep the per-item passes.
  const int64_t shfix = plk_opt(PLK_OPT_NTT_SHARED_FIX);
  bool anyfix = false;
  for (int j = 0; j < nj; j++) anyfix |= jobs.j[j].bfix != 0;
  WJobs cj = jobs;
  if (shfix > 1 || (shfix == 1 && !anyfix)) {
    WArrs sh{};
    int ns = 0;
    for (int q = 0; q < na; q++) {
      int uses = 0;
      for (int j = 0; j < nj; j++) uses += (jobs.j[j].A == arrs.a[q].d) + (!jobs.j[j].bfix && jobs.j[j].B == arrs.a[q].d);
      if (uses < 2) continue;
      sh.a[ns++] = arrs.a[q];
      for (int j = 0; j < nj; j++) {
        if (cj.j[j].A == arrs.a[q].d) cj.j[j].afix = 1;
        if (!jobs.j[j].bfix && cj.j[j].B == arrs.a[q].d) cj.j[j].bfix = 1;
      }
    }
    // (PLK_NTT_FIX_FILL) the launch runs ceil(ns tiles / resident) rounds of resident blocks: fill its
    // last round with operands used once, whose lo = 0 pass then leaves the centre items
    if (PLK_NTT_FIX_FILL && ns) {
      const uint32_t per = std::max<uint32_t>(1u, center_blocks() / std::max<uint32_t>(tiles, 1u));
      int extra = (int)(((uint32_t)ns + per - 1) / per * per) - ns;
      for (int q = arrs.derive ? 1 : 0; q < na && extra > 0 && ns < WT_MAX_ARRS; q++) {
        bool fixed = false;
        for (int t = 0; t < ns; t++) fixed |= sh.a[t].d == arrs.a[q].d;
        if (fixed) continue;
        sh.a[ns++] = arrs.a[q];
        extra--;
        for (int j = 0; j < nj; j++) {
          if (cj.j[j].A == arrs.a[q].d) cj.j[j].afix = 1;
          if (!jobs.j[j].bfix && cj.j[j].B == arrs.a[q].d) cj.j[j].bfix = 1;
        }
      }
    }
    if (ns) {
      log_launch<F>(3, TB, TB, k, ns, 1, ns);
      hipLaunchKernelGGL((wt_fixfwd_kernel<TB, wt_rc(TB), F>), dim3(tiles, ns), dim3(wt_ntc(TB)), 0, st, WPass{k, 0}, sh,
                         twf);
      PLK_HIP(hipGetLastError());
    }
  }
  WJobs ij = jobs;   // the inverse passes' jobs
  if (plk_opt(PLK_OPT_NTT_CENTER_SUM)) merge_groups(cj, ij, nj);
  const WSched sc = center_schedule(cj, nj, tiles, center_blocks());
  const uint32_t grid = (uint32_t)std::min<uint64_t>((uint64_t)tiles * sc.n, center_blocks());
  bool grp = false;
  for (int j = 0; j < nj; j++) grp |= cj.j[j].ncm > 0;
  if (grid) {
    int units = 0;
    for (int j = 0; j < nj; j++) units += center_units(cj, j);
    log_launch<F>(2, TB, TB, k, nj, 1, units);
    if (grp)
      hipLaunchKernelGGL((wt_center_kernel<TB, wt_rc(TB), F, true>), dim3(grid), dim3(wt_ntc(TB)), 0, st, WPass{k, 0},
                         cj, twf, sc);
    else
      hipLaunchKernelGGL((wt_center_kernel<TB, wt_rc(TB), F, false>), dim3(grid), dim3(wt_ntc(TB)), 0, st, WPass{k, 0},
                         cj, twf, sc);
    PLK_HIP(hipGetLastError());
  }
  const WTw twi = inv_wtw<F>(k);
  // the inverse passes' grid: the jobs that have any (sum-group members have none)
  WJobs ic{};
  int ni = 0;
  for (int j = 0; j < nj; j++)
    if (!ij.j[j].skip_inv) ic.j[ni++] = ij.j[j];
  WJobs later = ic;   // sum groups add their members in the FIRST inverse pass only
  for (int j = 0; j < ni; j++) later.j[j].S1 = later.j[j].S2 = nullptr;
  for (int i = np - 2; i >= 0; i--) {
    const WPass p{k, lo[i]};
    const WJobs& jj = i == np - 2 ? ic : later;
    rc = i == 0 ? inv_m<TB, true, F>(Ms[i], p, jj, ni, twi, ninv, st)
                : inv_m<TB, false, F>(Ms[i], p, jj, ni, twf, 0u, st);
    if (rc) return rc;
  }
  bool wrapped = false;
  for (int j = 0; j < ni; j++) wrapped |= ic.j[j].ntop > 0;
  if (wrapped && !PLK_NTT_WRAP_INLINE) {   // (after the last inverse pass's byte stores, on the same stream)
    hipLaunchKernelGGL(wrap_fix_kernel, dim3(ni), dim3(64), 0, st, ic, 1ull << k);
    PLK_HIP(hipGetLastError());
  }
  return PLK_OK;
}

// b's forward transform for WJob::bfix: the forward passes of a product (bytes in), then the
// center's lo = 0 pass stored in its register order
template <int TB, class F>
int wave_pretransform_t(const uint8_t* b8, uint64_t lb, int k, uint32_t* d, hipStream_t st) {
  const WTw twf = fwd_wtw<F>(k);
  int Ms[4];
  const int np = wave_plan(k, TB, Ms);
  int lo[4];
  for (int i = 0, top = k; i < np; i++) { lo[i] = top - Ms[i]; top = lo[i]; }
  WArrs arrs{};
  arrs.a[0] = WArr{d, b8, lb};
  for (int i = 0; i < np - 1; i++) {
    const WPass p{k, lo[i]};
    const int rc = i == 0 ? fwd_m<TB, true, F>(Ms[i], p, arrs, 1, twf, st) : fwd_m<TB, false, F>(Ms[i], p, arrs, 1, twf, st);
    if (rc) return rc;
  }
  hipLaunchKernelGGL((wt_fixfwd_kernel<TB, wt_rc(TB), F>), dim3((unsigned)((1ull << k) >> TB)), dim3(wt_ntc(TB)), 0, st,
                     WPass{k, 0}, arrs, twf);
  PLK_HIP(hipGetLastError());
  return PLK_OK;
}

template <int TB, class F>
int wave_ntt_t(const WJobs& jobs, const WArrs& arrs, int nj, int k, int inverse, hipStream_t st) {
  const PlkTwTables t = F::ADIC == f29::TWO_ADICITY ? plk_ntt_tables29() : plk_ntt_tables();
  int Ms[4];
  const int np = wave_plan(k, TB, Ms);
  int lo[4];
  for (int i = 0, top = k; i < np; i++) { lo[i] = top - Ms[i]; top = lo[i]; }
  for (int s = 0; s < np; s++) {
    const int i = inverse ? np - 1 - s : s;
    const WPass p{k, lo[i]};
    const int rc = inverse ? inv_m<TB, false, F>(Ms[i], p, jobs, nj, to_wtw(t, true), 0u, st)
                           : fwd_m<TB, false, F>(Ms[i], p, arrs, nj, fwd_wtw<F>(k), st);
    if (rc) return rc;
  }
  return PLK_OK;
}

}  // namespace

bool plk_wave_ntt_supported(int k) { return k > 12 && k <= bb::TWO_ADICITY; }

namespace {
template <class F>
int build_coltabs(int fi) {
  for (int k = COLT_MIN_K; k <= COLT_MAX_K; k++) {
    // (the scale: ntt.hip's N^-1 R^2 for a 2^k product)
    const uint32_t ninv = fi ? (uint32_t)((uint64_t)f29::hpow(1ull << k, f29::P - 2) * f29::R2 % f29::P)
                             : (uint32_t)((uint64_t)bb::hpow(1ull << k, bb::P - 2) * bb::R2 % bb::P);
    for (int s = 0; s < 2; s++) {
      const int dev = plk_cur_device();
      uint32_t*& t = s ? g_coli[dev][fi][k] : g_col[dev][fi][k];
      if (t || !two_pass(k)) continue;   // (three-pass plans take no table: fwd_wtw)
      PLK_HIP(hipMalloc((void**)&t, 4ull << k));
      const WTw tw = to_wtw(fi ? plk_ntt_tables29() : plk_ntt_tables(), false);
      const unsigned blocks = (unsigned)((1ull << k) / 256);
      const uint32_t sc = s ? ninv : 0u;
      if (tile_bits(k) == 13) hipLaunchKernelGGL((coltab_kernel<13, F>), dim3(blocks), dim3(256), 0, 0, t, k, tw, sc);
      else hipLaunchKernelGGL((coltab_kernel<12, F>), dim3(blocks), dim3(256), 0, 0, t, k, tw, sc);
      PLK_HIP(hipGetLastError());
    }
  }
  return PLK_OK;
}
}  // namespace

// 2 x 2 x 64 MB of column tables (BabyBear and F29, 2^13 .. 2^23 points; forward and scaled
// inverse), built on the device
int plk_wave_init_coltabs(void) {
  int rc = build_coltabs<FBB>(0);
  if (!rc) rc = build_coltabs<F29>(1);
  if (!rc) PLK_HIP(hipDeviceSynchronize());
  return rc;
}
// the current device's column tables
void plk_wave_free_coltabs(void) {
  const int dev = plk_cur_device();
  for (auto* g : {&g_col[dev], &g_coli[dev]})
    for (auto& f : *g)
      for (auto& t : f) {
        (void)hipFree(t);
        t = nullptr;
      }
}

int plk_wave_poly_mul_batch_launch(const WJob* jobs, int nj, int k, int field, uint32_t ninv, hipStream_t st) {
  for (int j0 = 0; j0 < nj; j0 += WT_MAX_JOBS) {
    const int m = nj - j0 < WT_MAX_JOBS ? nj - j0 : WT_MAX_JOBS;
    WJobs w{};
    for (int i = 0; i < m; i++) w.j[i] = jobs[j0 + i];
    const bool t13 = tile_bits(k) == 13;
    const int rc = field == 1 ? (t13 ? wave_poly_mul_t<13, F29>(w, m, k, ninv, st) : wave_poly_mul_t<12, F29>(w, m, k, ninv, st))
                              : (t13 ? wave_poly_mul_t<13, FBB>(w, m, k, ninv, st) : wave_poly_mul_t<12, FBB>(w, m, k, ninv, st));
    if (rc) return rc;
  }
  return PLK_OK;
}

int plk_wave_pretransform(const uint8_t* b8, uint64_t lb, int k, int field, uint32_t* d_out, hipStream_t st) {
  if (!plk_wave_ntt_supported(k) || lb == 0 || lb > (1ull << k)) {
    plk_set_error("pretransform: %llu coefficients at 2^%d", (unsigned long long)lb, k);
    return PLK_ERR_ARG;
  }
  const bool t13 = tile_bits(k) == 13;
  return field == 1 ? (t13 ? wave_pretransform_t<13, F29>(b8, lb, k, d_out, st) : wave_pretransform_t<12, F29>(b8, lb, k, d_out, st))
                    : (t13 ? wave_pretransform_t<13, FBB>(b8, lb, k, d_out, st) : wave_pretransform_t<12, FBB>(b8, lb, k, d_out, st));
}

// batch independent in-place transforms of 2^k points: array i at d + i 2^k, <= 12 per launch
int plk_wave_ntt_launch(uint32_t* d, int k, int batch, int inverse, int field, hipStream_t st) {
  for (int j0 = 0; j0 < batch; j0 += WT_MAX_JOBS) {
    const int m = batch - j0 < WT_MAX_JOBS ? batch - j0 : WT_MAX_JOBS;
    WJobs w{};
    WArrs a{};
    for (int i = 0; i < m; i++) {
      w.j[i].A = w.j[i].C = a.a[i].d = d + ((uint64_t)(j0 + i) << k);
    }
    const bool t13 = tile_bits(k) == 13;
    const int rc = field == 1 ? (t13 ? wave_ntt_t<13, F29>(w, a, m, k, inverse, st) : wave_ntt_t<12, F29>(w, a, m, k, inverse, st))
                              : (t13 ? wave_ntt_t<13, FBB>(w, a, m, k, inverse, st) : wave_ntt_t<12, FBB>(w, a, m, k, inverse, st));
    if (rc) return rc;
  }
  return PLK_OK;
}

extern "C" int plk_ntt_launch_log(int32_t* out, int cap) {
  std::lock_guard<std::mutex> lk(g_log_mu);
  const int n = (int)std::min<size_t>(g_log.size(), cap > 0 ? (size_t)cap : 0);
  for (int i = 0; i < n && out; i++) {
    const LaunchRec& r = g_log[i];
    const int32_t v[8] = {r.kind, r.tb, r.m, r.k, r.n, r.per_block, r.units, r.field};
    for (int f = 0; f < 8; f++) out[8 * i + f] = v[f];
  }
  g_log.clear();
  return n;
}
