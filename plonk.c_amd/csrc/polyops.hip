// The polynomial and matrix ops around the hot path on gfx950:
//
//   poly_eval        src/poly.h:265-272   Horner over GF(17) on raw bytes
//   poly_divide      src/poly.h:124-177   long division num = quot * den + rem
//   matrix_mul       src/matrix.h:79-96   (interpolate_at_h, src/plonk.h:162-195)
//   matrix_inv       src/matrix.h:100-176 (plonk_new's Vandermonde inverse, src/plonk.h:105-113)
//
// Every op reproduces the reference's BYTE arithmetic, including non-canonical coefficient
// bytes (HF values >= 17): hf_add is a uint8 sum with one conditional subtract, hf_sub an int8
// difference with one conditional add, hf_mul (a * b) % 17 (src/hf.h:79-116).  The parallel
// paths hold on canonical inputs (or, for poly_eval, on inputs where no uint8 sum can wrap);
// the kernels detect the other inputs and run the reference's loop serially on the device.
#include "plk_device.h"
#include "plk_internal.h"

#include <stdlib.h>
#include <string.h>

namespace {

constexpr uint32_t HP = 17;
__constant__ uint8_t c_hinv17[17] = {0, 1, 9, 6, 13, 7, 3, 5, 15, 2, 12, 14, 10, 4, 11, 8, 16};

// the reference's raw byte ops (src/hf.h:79-116)
__device__ __forceinline__ uint32_t raw_add(uint32_t a, uint32_t b) {
  const uint32_t s = (a + b) & 0xFFu;
  return s >= HP ? s - HP : s;
}
__device__ __forceinline__ uint32_t raw_sub(uint32_t a, uint32_t b) {
  int8_t d = (int8_t)((int)(int8_t)a - (int)(int8_t)b);
  if (d < 0) d = (int8_t)(d + (int)HP);
  return (uint8_t)d;
}
__device__ __forceinline__ uint32_t raw_mul(uint32_t a, uint32_t b) { return a * b % HP; }

// block-wide sum of per-thread values (every thread calls; result valid in thread 0)
template <int NT>
__device__ __forceinline__ uint32_t block_sum(uint32_t v) {
  __shared__ uint32_t ws[NT / PLK_WAVE];
  v = plk_wave_sum(v);
  if ((threadIdx.x & (PLK_WAVE - 1)) == 0) ws[threadIdx.x / PLK_WAVE] = v;
  __syncthreads();
  uint32_t t = 0;
  if (threadIdx.x == 0)
#pragma unroll
    for (int w = 0; w < NT / PLK_WAVE; w++) t += ws[w];
  return t;
}

// ---------------------------------------------------------------------------------------
// poly_eval.  Horner: y = 0; for i = len-1 .. 0: y = hf_add(hf_mul(y, x), c_i).  hf_mul
// reduces mod 17, so only the residue of an intermediate y matters -- except that hf_add's
// uint8 sum can wrap (256 = 1 mod 17 changes the residue), which needs c_i >= 240.  With no
// such c_i at i >= 1, y_1 = S = sum_{i>=1} c_i x^(i-1) (mod 17), and the output is the exact
// byte hf_add((S x) % 17, c_0).  x^e = x^(e mod 16) for x != 0 (mod 17).  A job with a
// c_i >= 240 (i >= 1) is re-run by its last block with the reference's loop.
// ---------------------------------------------------------------------------------------
constexpr int EVAL_NT = 256;
struct EvalJobs {
  const uint8_t* p[PLK_EVAL_MAX_JOBS];
  uint64_t len[PLK_EVAL_MAX_JOBS];
  uint8_t x[PLK_EVAL_MAX_JOBS];
};

__global__ __launch_bounds__(EVAL_NT) void eval_batch_kernel(EvalJobs J, uint8_t* __restrict__ y,
                                                             unsigned long long* __restrict__ tick) {
  const int job = blockIdx.y;
  const uint8_t* p = J.p[job];
  const uint64_t len = J.len[job];
  const uint32_t xm = J.x[job] % HP;
  // pw[i mod 16] = x^(i - 1) for i >= 1 (x = 0: only i = 1 contributes)
  uint32_t pw[16];
  {
    uint32_t e = 1;   // x^0
#pragma unroll
    for (int t = 1; t <= 16; t++) {
      pw[t & 15] = xm == 0 ? (t == 1 ? 1u : 0u) : e;
      e = e * xm % HP;
    }
  }
  uint32_t acc = 0, bad = 0;
  const uint64_t chunks = (len + 15) >> 4;
  const bool vec = ((uintptr_t)p & 15) == 0;
  for (uint64_t c = (uint64_t)blockIdx.x * EVAL_NT + threadIdx.x; c < chunks; c += (uint64_t)gridDim.x * EVAL_NT) {
    const uint64_t i0 = c << 4;
    uint32_t w[4];
    if (vec && i0 + 16 <= len) {
      const uint4 v = *reinterpret_cast<const uint4*>(p + i0);
      w[0] = v.x; w[1] = v.y; w[2] = v.z; w[3] = v.w;
    } else {
#pragma unroll
      for (int q = 0; q < 4; q++) w[q] = 0;
      for (int k = 0; k < 16; k++)
        if (i0 + k < len) w[k >> 2] |= (uint32_t)p[i0 + k] << (8 * (k & 3));
    }
#pragma unroll
    for (int k = 0; k < 16; k++) {
      const uint32_t b = (w[k >> 2] >> (8 * (k & 3))) & 0xFFu;
      const bool live = i0 + k > 0;           // c_0 is added exactly at the end
      acc += live ? b * pw[k] : 0u;           // (i0 + k) mod 16 = k; < 2^20 per chunk
      bad |= (live && b >= 240u) ? 1u : 0u;
    }
    acc %= HP;
  }
  const uint32_t s = block_sum<EVAL_NT>(acc % HP);
  const uint32_t anybad = __syncthreads_or(bad);
  if (threadIdx.x != 0) return;
  const unsigned long long add = (unsigned long long)(s % HP) | (1ull << 32) | ((unsigned long long)(anybad != 0) << 48);
  const unsigned long long old = atomicAdd(&tick[job * 16], add);
  if (((old >> 32) & 0xFFFFull) != gridDim.x - 1) return;
  const unsigned long long tot = old + add;
  atomicExch(&tick[job * 16], 0ull);
  uint32_t out = 0;
  if ((tot >> 48) == 0) {
    const uint32_t S = (uint32_t)(tot & 0xFFFFFFFFull) % HP;
    out = len ? raw_add(S * xm % HP, p[0]) : 0u;
  } else {   // the reference's loop, exactly
    const uint32_t xr = J.x[job];
    for (uint64_t i = len; i-- > 0;) out = raw_add(raw_mul(out, xr), p[i]);
  }
  y[job] = (uint8_t)out;
}

// ---------------------------------------------------------------------------------------
// poly_divide.  The reference's loop (for i = nl-1 .. dl-1: c = rem[i] * inv(lead);
// q[i-dl+1] = c; rem[i-j] -= c den[dl-1-j] for j < dl) on raw bytes, one thread: the general
// divisor and non-canonical inputs.
// ---------------------------------------------------------------------------------------
// The reference's loop (src/poly.h:124-177) on raw bytes, one thread.  den == nullptr: the
// binomial divisor lead x^(dl-1) + d0 given by its two bytes (the gated re-run behind the chain
// scans: no host-to-device copy of a mostly-zero divisor per call).
// The running remainder lives in the workspace (nl bytes); the caller's rem receives its first
// min(dl - 1, nl) bytes (the size plk_poly_divide_dev documents).
__device__ void serial_divide(const uint8_t* __restrict__ num, uint64_t nl, const uint8_t* __restrict__ den, uint64_t dl,
                              uint32_t d0, uint32_t lead, uint8_t* __restrict__ q, uint64_t qcap,
                              uint8_t* __restrict__ rem, uint64_t rl, uint8_t* __restrict__ run) {
  for (uint64_t i = 0; i < qcap; i++) q[i] = 0;
  for (uint64_t i = 0; i < nl; i++) run[i] = num[i];
  auto den_at = [&](uint64_t i) -> uint32_t { return den ? den[i] : (i == 0 ? d0 : (i == dl - 1 ? lead : 0u)); };
  const uint32_t inv = c_hinv17[den_at(dl - 1)];   // lead < 17 (host-checked)
  for (uint64_t i = nl; i-- > dl - 1;) {
    const uint32_t c = raw_mul(run[i], inv);
    q[i - (dl - 1)] = (uint8_t)c;
    // every j, zero divisor bytes included: hf_sub of raw bytes normalises as the reference does
    for (uint64_t j = 0; j < dl; j++) run[i - j] = (uint8_t)raw_sub(run[i - j], raw_mul(c, den_at(dl - 1 - j)));
  }
  for (uint64_t i = 0; i < rl; i++) rem[i] = run[i];
}

__device__ __forceinline__ uint32_t fin_block_max(uint32_t v, uint32_t* red) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v = max(v, (uint32_t)__shfl_xor(v, off, PLK_WAVE));
  __syncthreads();
  if ((threadIdx.x & (PLK_WAVE - 1)) == 0) red[threadIdx.x / PLK_WAVE] = v;
  __syncthreads();
  uint32_t m = 0;
  for (int w = 0; w < (int)(blockDim.x / PLK_WAVE); w++) m = max(m, red[w]);
  return m;
}
// index + 1 of the last non-zero byte of p[0, len) (0: all zero), scanning back 16 KiB at a time
__device__ uint32_t fin_trim(const uint8_t* __restrict__ p, uint64_t len, uint32_t* red) {
  constexpr int64_t CH = 16384;
  for (int64_t end = (int64_t)len; end > 0; end -= CH) {
    const int64_t start = end > CH ? end - CH : 0;
    uint32_t last = 0;
    for (int64_t i = start + threadIdx.x; i < end; i += blockDim.x)
      if (p[i]) last = max(last, (uint32_t)(i + 1));
    last = fin_block_max(last, red);
    if (last) return last;
  }
  return 0;
}

// ONE launch after the division kernels: the reference's loop when it is needed (mode 1: always,
// the divisor copied to the device; mode 2: only when the chain scans flagged non-canonical
// numerator bytes, binomial divisor by its two bytes), then the trimmed lengths of q and rem
// (src/poly.h:158-170) -- three launches (serial re-run + two trims) folded into one.
__global__ __launch_bounds__(1024) void div_finish_kernel(const uint8_t* __restrict__ num, uint64_t nl,
                                                         const uint8_t* __restrict__ den, uint64_t dl, uint32_t d0,
                                                         uint32_t lead, uint8_t* __restrict__ q, uint64_t ql,
                                                         uint8_t* __restrict__ rem, uint64_t rl, int mode,
                                                         const uint32_t* __restrict__ gate, uint8_t* __restrict__ scratch,
                                                         uint32_t* __restrict__ lens) {
  __shared__ uint32_t red[16];
  const bool run = mode == 1 || (mode == 2 && *gate != 0);   // uniform
  if (run && threadIdx.x == 0) serial_divide(num, nl, den, dl, d0, lead, q, ql, rem, rl, scratch);
  __syncthreads();   // thread 0's global writes are visible to the block after the barrier
  const uint32_t lq = fin_trim(q, ql, red);
  const uint32_t lr = rl ? fin_trim(rem, rl, red) : 0u;
  if (threadIdx.x == 0) {
    lens[0] = lq;
    lens[1] = lr;
  }
}

// Divisor lead x^m + d0 (every other coefficient zero; m = dl - 1 >= 1), canonical bytes.  The
// loop gives q[k] = inv (num[k+m] - d0 q[k+m]) = v_k + A q[k+m] with A = -d0 inv, v_k = inv
// num[k+m]: m independent chains k = r, r + m, r + 2m, ...  and rem[t] = num[t] - d0 q[t]
// (t < m).  Short chains: one thread walks a chain from its top.
struct Binom {
  const uint8_t* num;
  uint64_t nl, m, lq;      // lq = nl - m quotient coefficients
  uint32_t inv, d0;
  uint8_t* q;
  uint8_t* rem;
  uint32_t* flag;          // set when some num byte is not canonical (serial path re-runs)
};

__global__ __launch_bounds__(256) void div_binom_short_kernel(Binom B) {
  const uint64_t r = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= B.m) return;
  const uint32_t A = (HP - B.d0 * B.inv % HP) % HP;
  uint32_t prev = 0, bad = 0;
  if (r < B.lq) {
    const uint64_t cnt = (B.lq - 1 - r) / B.m + 1;
    for (uint64_t t = cnt; t-- > 0;) {
      const uint64_t k = r + t * B.m;
      const uint32_t b = B.num[k + B.m];
      bad |= b >= HP;
      prev = (b * B.inv + A * prev) % HP;
      B.q[k] = (uint8_t)prev;
    }
  }
  if (r < B.nl) {   // remainder coefficient r (r < m); prev = q[r], 0 when r has no quotient
    const uint32_t b = B.num[r];
    bad |= b >= HP;
    B.rem[r] = (uint8_t)((b + (HP - B.d0) * prev) % HP);
  }
  if (bad) atomicOr(B.flag, 1u);
}

// Long chains (m small, e.g. the linear divisors x - z of src/plonk.h:604-613): with A != 0,
// q_p = A^-p sum_{s >= p} A^s v_s along a chain (positions p; A^16 = 1), a suffix sum --
// two phases over blocks of SCAN_B positions: block aggregates, then each block reduces the
// aggregates after it and scans within itself.  A = 0 needs no scan (q = v).
constexpr int SCAN_T = 256, SCAN_E = 16, SCAN_B = SCAN_T * SCAN_E;

__device__ __forceinline__ void pow16(uint32_t a, uint32_t (&pw)[16]) {
  pw[0] = 1;
#pragma unroll
  for (int j = 1; j < 16; j++) pw[j] = pw[j - 1] * a % HP;
}

// chain r = blockIdx.y + y0, positions [blockIdx.x SCAN_B, +SCAN_B)
__global__ __launch_bounds__(SCAN_T) void div_binom_sums_kernel(Binom B, uint64_t y0, uint64_t nblk,
                                                                uint32_t* __restrict__ bsum) {
  const uint64_t r = y0 + blockIdx.y;
  const uint64_t len = (B.lq - 1 - r) / B.m + 1;   // chain length (r < min(m, lq): host)
  const uint32_t A = (HP - B.d0 * B.inv % HP) % HP;
  uint32_t pw[16];
  pow16(A, pw);
  const uint64_t p0 = (uint64_t)blockIdx.x * SCAN_B + (uint64_t)threadIdx.x * SCAN_E;
  uint32_t acc = 0, bad = 0;
#pragma unroll
  for (int e = 0; e < SCAN_E; e++) {
    const uint64_t p = p0 + e;
    if (p < len) {
      const uint32_t b = B.num[r + (p + 1) * B.m];
      bad |= b >= HP;
      acc += b * B.inv % HP * pw[p & 15];
    }
  }
  const uint32_t t = block_sum<SCAN_T>(acc % HP);
  if (__syncthreads_or(bad) && threadIdx.x == 0) atomicOr(B.flag, 1u);
  if (threadIdx.x == 0) bsum[blockIdx.y * nblk + blockIdx.x] = t % HP;
}

__global__ __launch_bounds__(SCAN_T) void div_binom_apply_kernel(Binom B, uint64_t y0, uint64_t nblk,
                                                                 const uint32_t* __restrict__ bsum) {
  __shared__ uint32_t wtot[SCAN_T / PLK_WAVE];
  __shared__ uint32_t carry_s;
  const uint64_t r = y0 + blockIdx.y;
  const uint64_t len = (B.lq - 1 - r) / B.m + 1;
  const uint32_t A = (HP - B.d0 * B.inv % HP) % HP;
  uint32_t pw[16], ipw[16];
  pow16(A, pw);
  pow16(c_hinv17[A], ipw);
  // carry: aggregates of the blocks after this one
  if (threadIdx.x < PLK_WAVE) {
    uint32_t c = 0;
    for (uint64_t b = blockIdx.x + 1 + threadIdx.x; b < nblk; b += PLK_WAVE) c += bsum[blockIdx.y * nblk + b];
    c = plk_wave_sum(c % HP);
    if (threadIdx.x == 0) carry_s = c % HP;
  }
  const uint64_t p0 = (uint64_t)blockIdx.x * SCAN_B + (uint64_t)threadIdx.x * SCAN_E;
  uint32_t v[SCAN_E], tot = 0;
#pragma unroll
  for (int e = 0; e < SCAN_E; e++) {
    const uint64_t p = p0 + e;
    v[e] = p < len ? B.num[r + (p + 1) * B.m] * B.inv % HP : 0u;
    tot += A ? v[e] * pw[p & 15] : 0u;
  }
  tot %= HP;
  // exclusive suffix over threads: sum of the totals of threads after this one
  const int lane = threadIdx.x & (PLK_WAVE - 1), wave = threadIdx.x / PLK_WAVE;
  uint32_t suf = tot;
#pragma unroll
  for (int d = 1; d < PLK_WAVE; d <<= 1) {
    const uint32_t o = __shfl_down(suf, d, PLK_WAVE);
    if (lane + d < PLK_WAVE) suf += o;
  }
  if (lane == 0) wtot[wave] = suf % HP;
  __syncthreads();
  uint32_t after = (suf - tot) % HP + carry_s;   // this wave's threads after me, + later blocks
  for (int w = wave + 1; w < SCAN_T / PLK_WAVE; w++) after += wtot[w];
  after %= HP;
  uint32_t run = after;   // sum_{s > p} A^s v_s
  uint32_t q0 = 0;
#pragma unroll
  for (int e = SCAN_E - 1; e >= 0; e--) {
    const uint64_t p = p0 + e;
    if (p < len) {
      uint32_t qv;
      if (A) {
        run = (run + v[e] * pw[p & 15]) % HP;
        qv = run * ipw[p & 15] % HP;
      } else {
        qv = v[e];
      }
      B.q[r + p * B.m] = (uint8_t)qv;
      if (p == 0) q0 = qv;
    }
  }
  if (p0 == 0 && r < B.nl) {
    const uint32_t b = B.num[r];
    if (b >= HP) atomicOr(B.flag, 1u);
    B.rem[r] = (uint8_t)((b % HP + (HP - B.d0) * q0) % HP);
  }
}

// divisor of length 1 (m = 0): q = num * inv(lead) bytewise, no remainder coefficients
__global__ __launch_bounds__(256) void div_const_kernel(const uint8_t* __restrict__ num, uint64_t nl, uint32_t inv,
                                                        uint8_t* __restrict__ q) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nl; i += (uint64_t)gridDim.x * blockDim.x)
    q[i] = (uint8_t)raw_mul(num[i], inv);
}

// ---------------------------------------------------------------------------------------
// matrices (row-major bytes, src/matrix.h).  matrix_mul: sum = hf_add(sum, hf_mul(a, b)) per
// element (one thread each).  matrix_inv: Gauss-Jordan on [M | I] exactly as
// matrix_gauss_jordan (src/matrix.h:100-147) -- pivot search, swaps, normalisation and
// elimination in the reference's order, one workgroup (n is |H| <= 17 in GF(17)).
// ---------------------------------------------------------------------------------------
__global__ void matrix_mul_kernel(const uint8_t* __restrict__ a, const uint8_t* __restrict__ b, uint64_t m, uint64_t k,
                                  uint64_t n, uint8_t* __restrict__ out) {
  for (uint64_t e = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; e < m * n; e += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t i = e / n, j = e % n;
    uint32_t s = 0;
    for (uint64_t t = 0; t < k; t++) s = raw_add(s, raw_mul(a[i * k + t], b[t * n + j]));
    out[e] = (uint8_t)s;
  }
}

// aug: n x 2n workspace (global); one block of 256 threads; columns in parallel per row op
__global__ __launch_bounds__(256) void matrix_inv_kernel(const uint8_t* __restrict__ mat, uint64_t n,
                                                         uint8_t* __restrict__ aug, uint8_t* __restrict__ out) {
  const uint64_t cols = 2 * n;
  for (uint64_t e = threadIdx.x; e < n * cols; e += blockDim.x) {
    const uint64_t i = e / cols, j = e % cols;
    aug[e] = j < n ? mat[i * n + j] : (j - n == i ? 1 : 0);
  }
  __syncthreads();
  __shared__ uint64_t s_i, s_lead;
  __shared__ int s_stop;
  uint64_t lead = 0;
  for (uint64_t r = 0; r < n; r++) {
    if (threadIdx.x == 0) {   // pivot search (src/matrix.h:108-118), serial as in the reference
      int stop = lead >= cols;
      uint64_t i = r;
      while (!stop && aug[i * cols + lead] == 0) {
        i++;
        if (i == n) {
          i = r;
          lead++;
          if (lead == cols) stop = 1;
        }
      }
      s_i = i;
      s_lead = lead;
      s_stop = stop;
    }
    __syncthreads();
    if (s_stop) break;
    lead = s_lead;
    const uint64_t i = s_i;
    if (i != r)
      for (uint64_t k = threadIdx.x; k < cols; k += blockDim.x) {
        const uint8_t t = aug[i * cols + k];
        aug[i * cols + k] = aug[r * cols + k];
        aug[r * cols + k] = t;
      }
    __syncthreads();
    const uint32_t div = aug[r * cols + lead];
    __syncthreads();
    if (div != 0)   // hf_div(value, div) = value * inv(div); div < 17 (host-checked bytes)
      for (uint64_t k = threadIdx.x; k < cols; k += blockDim.x)
        aug[r * cols + k] = (uint8_t)raw_mul(aug[r * cols + k], c_hinv17[div]);
    __syncthreads();
    // eliminate every other row (src/matrix.h:130-143): rows are independent given row r, so in
    // parallel; each row's multiplier is captured before its update
    __shared__ uint8_t mults[1024];
    for (uint64_t ii = threadIdx.x; ii < n; ii += blockDim.x) mults[ii] = aug[ii * cols + lead];
    __syncthreads();
    for (uint64_t e = threadIdx.x; e < n * cols; e += blockDim.x) {
      const uint64_t ii = e / cols, k = e % cols;
      if (ii == r) continue;
      aug[e] = (uint8_t)raw_sub(aug[e], raw_mul(aug[r * cols + k], mults[ii]));
    }
    __syncthreads();
    lead++;
  }
  __syncthreads();
  for (uint64_t e = threadIdx.x; e < n * n; e += blockDim.x) out[e] = aug[(e / n) * cols + n + e % n];
}

}  // namespace

// ------------------------------------------------------------------------------ launchers
int plk_poly_eval_batch_launch(const uint8_t* const* polys, const uint64_t* lens, const uint8_t* xs, int nj,
                               uint8_t* d_y, void* d_tick, hipStream_t st) {
  if (nj < 1 || nj > PLK_EVAL_MAX_JOBS) {
    plk_set_error("poly_eval batch: %d jobs (1..%d)", nj, PLK_EVAL_MAX_JOBS);
    return PLK_ERR_ARG;
  }
  EvalJobs J{};
  uint64_t mx = 0;
  for (int i = 0; i < nj; i++) {
    if (!polys[i] && lens[i]) {
      plk_set_error("poly_eval batch: job %d has a NULL polynomial", i);
      return PLK_ERR_ARG;
    }
    J.p[i] = polys[i];
    J.len[i] = lens[i];
    J.x[i] = xs[i];
    mx = lens[i] > mx ? lens[i] : mx;
  }
  // blocks per job: one per 64 KiB, at most 64 (the finish's ticket sums 16 bits)
  uint64_t nb = (mx + 65535) >> 16;
  nb = nb < 1 ? 1 : (nb > 64 ? 64 : nb);
  hipLaunchKernelGGL(eval_batch_kernel, dim3((unsigned)nb, nj), dim3(EVAL_NT), 0, st, J, d_y,
                     (unsigned long long*)d_tick);
  PLK_HIP(hipGetLastError());
  return PLK_OK;
}

size_t plk_poly_divide_workspace_bytes(uint64_t nl, uint64_t dl) {
  // den copy + flag/length words + scan block aggregates (long chains)
  const uint64_t m = dl ? dl - 1 : 0;
  const uint64_t lq = nl >= dl ? nl - m : 0;
  const uint64_t chains = m < lq ? m : lq;
  const uint64_t len = chains ? (lq + m - 1) / (m ? m : 1) : 0;
  const uint64_t nblk = (len + SCAN_B - 1) / SCAN_B;
  return 256 + ((dl + 15) & ~15ull) + 4 * (chains * nblk + 16) + ((nl + 15) & ~15ull);   // + the serial remainder
}

// Classifies the divisor on the host (den is a host array; the kernels get its bytes by value or
// in d_work), enqueues the division; d_lens[0] / d_lens[1] receive the index + 1 of the last
// non-zero quotient / remainder byte (0 if none) over the untrimmed lengths
// ql = nl >= dl ? nl - dl + 1 : 1 and rl = min(dl - 1, nl).
int plk_poly_divide_launch(const uint8_t* d_num, uint64_t nl, const uint8_t* den, uint64_t dl, uint8_t* d_q,
                           uint8_t* d_rem, uint32_t* d_lens, void* d_work, hipStream_t st) {
  if (!den || dl == 0) {
    plk_set_error("Division by zero polynomial in poly_divide");
    return PLK_ERR_ARG;
  }
  bool zero = true;
  for (uint64_t i = 0; i < dl && zero; i++) zero = den[i] == 0;
  if (zero) {
    plk_set_error("Division by zero polynomial in poly_divide");
    return PLK_ERR_ARG;
  }
  const uint32_t lead = den[dl - 1];
  if (lead >= HP) {   // the reference indexes hf_inverses[17] out of bounds: undefined
    plk_set_error("poly_divide: divisor lead byte %u is not a GF(17) value (reference behaviour undefined)", lead);
    return PLK_ERR_RANGE;
  }
  if (nl && !d_num) {
    plk_set_error("poly_divide: NULL numerator");
    return PLK_ERR_ARG;
  }
  const uint64_t m = dl - 1;
  const uint64_t ql = nl >= dl ? nl - dl + 1 : 1;
  const uint64_t rl = m < nl ? m : nl;
  uint8_t* w = (uint8_t*)d_work;
  uint32_t* flag = (uint32_t*)w;           // [0] non-canonical flag
  uint8_t* d_den = w + 256;
  uint32_t* bsum = (uint32_t*)(w + 256 + ((dl + 15) & ~15ull));
  uint8_t* scratch = w + plk_poly_divide_workspace_bytes(nl, dl) - ((nl + 15) & ~15ull);   // last nl bytes
  PLK_HIP(hipMemsetAsync(flag, 0, 16, st));
  bool canonical_den = true;
  bool binom = true;
  for (uint64_t i = 0; i < dl; i++) {
    canonical_den &= den[i] < HP;
    if (i > 0 && i + 1 < dl && den[i]) binom = false;
  }
  const uint32_t inv = [](uint32_t a) {
    static const uint8_t t[17] = {0, 1, 9, 6, 13, 7, 3, 5, 15, 2, 12, 14, 10, 4, 11, 8, 16};
    return (uint32_t)t[a];
  }(lead);
  bool serial = !canonical_den || !binom || lead == 0;
  if (!serial) {
    if (nl < dl) {
      // no loop step: q = {0}, rem = num[0 .. rl) -- parallel path still checks num's bytes
      PLK_HIP(hipMemsetAsync(d_q, 0, 1, st));
      if (rl) PLK_HIP(hipMemcpyAsync(d_rem, d_num, rl, hipMemcpyDeviceToDevice, st));
    } else if (m == 0) {
      const uint64_t b = (nl + 255) / 256;
      hipLaunchKernelGGL(div_const_kernel, dim3((unsigned)(b > 8192 ? 8192 : b)), dim3(256), 0, st, d_num, nl, inv, d_q);
      PLK_HIP(hipGetLastError());
    } else {
      Binom B{d_num, nl, m, nl - m, inv, den[0], d_q, d_rem, flag};
      const uint64_t lq = nl - m;
      const uint64_t chains = m < lq ? m : lq;
      const uint64_t len = (lq + m - 1) / m;   // longest chain
      if (len <= 4096) {
        const uint64_t b = (m + 255) / 256;
        hipLaunchKernelGGL(div_binom_short_kernel, dim3((unsigned)b), dim3(256), 0, st, B);
        PLK_HIP(hipGetLastError());
      } else {
        const uint64_t nblk = (len + SCAN_B - 1) / SCAN_B;
        for (uint64_t y0 = 0; y0 < chains; y0 += 65535) {
          const uint64_t ny = chains - y0 < 65535 ? chains - y0 : 65535;
          hipLaunchKernelGGL(div_binom_sums_kernel, dim3((unsigned)nblk, (unsigned)ny), dim3(SCAN_T), 0, st, B, y0,
                             nblk, bsum + y0 * nblk);
          PLK_HIP(hipGetLastError());
          hipLaunchKernelGGL(div_binom_apply_kernel, dim3((unsigned)nblk, (unsigned)ny), dim3(SCAN_T), 0, st, B,
                             y0, nblk, bsum + y0 * nblk);
          PLK_HIP(hipGetLastError());
        }
      }
    }
  }
  // a divisor outside the parallel forms, or (binomial path) non-canonical numerator bytes: the
  // reference's loop.  (m = 0 and nl < dl are exact for any bytes: hf_mul reduces, copies copy.)
  const bool gated = !serial && nl >= dl && m > 0;
  if (serial) PLK_HIP(hipMemcpyAsync(d_den, den, dl, hipMemcpyHostToDevice, st));
  hipLaunchKernelGGL(div_finish_kernel, dim3(1), dim3(1024), 0, st, d_num, nl, serial ? d_den : nullptr, dl,
                     (uint32_t)den[0], lead, d_q, ql, d_rem, rl, serial ? 1 : (gated ? 2 : 0), flag, scratch, d_lens);
  PLK_HIP(hipGetLastError());
  return PLK_OK;
}

int plk_matrix_mul_launch(const uint8_t* d_a, uint64_t m, uint64_t k, const uint8_t* d_b, uint64_t n, uint8_t* d_out,
                          hipStream_t st) {
  const uint64_t e = m * n;
  if (!e) return PLK_OK;
  const uint64_t b = (e + 255) / 256;
  hipLaunchKernelGGL(matrix_mul_kernel, dim3((unsigned)(b > 4096 ? 4096 : b)), dim3(256), 0, st, d_a, d_b, m, k, n,
                     d_out);
  PLK_HIP(hipGetLastError());
  return PLK_OK;
}

int plk_matrix_inv_launch(const uint8_t* d_mat, uint64_t n, uint8_t* d_aug, uint8_t* d_out, hipStream_t st) {
  if (n > 1024) {
    plk_set_error("matrix_inv: n = %llu (max 1024)", (unsigned long long)n);
    return PLK_ERR_RANGE;
  }
  if (!n) return PLK_OK;
  hipLaunchKernelGGL(matrix_inv_kernel, dim3(1), dim3(256), 0, st, d_mat, n, d_aug, d_out);
  PLK_HIP(hipGetLastError());
  return PLK_OK;
}
