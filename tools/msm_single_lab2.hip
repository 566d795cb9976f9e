// Single-MSM lab, part 2 (tuning aid, not part of the product): variants of the library's
// one-pass kernel for ONE 2^22-point MSM per launch, one 16-point group per thread:
//   ORDER 0  loads q0 q1 q2 s, each point's term computed in point order (the library)
//   ORDER 1  loads s q0 q1 q2: the terms of points 0-4 wait only for s and q0, ...
//   ORDER 2  loads q0 q1 q2 s: all lookups first (chunked by the word they need), the
//            multiplies by the scalars last
//   EXPLDS   the EXP table (102 words) is staged in LDS with the lookup table, so the last
//            finisher's point lookup is not a dependent global load at the end of the launch
// Inputs are random bytes (every point flagged irregular: the timing is what matters here,
// with random lookup indices as in real inputs), rotated over 40 sets (640 MiB > the 256 MiB
// Infinity Cache).
//
//   hipcc -O3 --offload-arch=gfx950 -std=c++17 tools/msm_single_lab2.hip -o tools/msm_single_lab2
//   rocprofv3 --kernel-trace --stats -d out -o run -- ./tools/msm_single_lab2
#include "../plonk.c_amd/csrc/msm.hip"

#include <stdarg.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include <functional>
#include <string>
#include <vector>

void plk_set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vfprintf(stderr, fmt, ap);
  va_end(ap);
  fputc('\n', stderr);
}

#define CK(x)                                                         \
  do {                                                                \
    hipError_t e = (x);                                               \
    if (e != hipSuccess) {                                            \
      printf("%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e)); \
      exit(1);                                                        \
    }                                                                 \
  } while (0)

namespace lab2 {

template <int C, int J, int ABL = 0>
__device__ __forceinline__ uint32_t dval(const uint32_t (&w)[12], const uint32_t* tab, uint32_t lane4) {
  const uint32_t k = point_bytes<J>(w);
  const uint32_t idx = (k >> 16) & 0x1FFu;
  if (ABL & 1) return (((idx << copy_shift<C>()) | lane4) * 0x9E3779B1u) - k;
  const uint32_t e = *reinterpret_cast<const uint32_t*>(reinterpret_cast<const char*>(tab) +
                                                        ((idx << copy_shift<C>()) | lane4));
  return e - k;
}

template <int NT, int C, int ORDER, bool EXPLDS, int SH = 8, bool HALF = false, int ABL = 0, int LATE = 0>
__global__ __launch_bounds__(NT) void k_v(const uint8_t* pts, const uint8_t* sc, PlkMsmResult* res,
                                          unsigned long long* shw) {
  __shared__ __attribute__((aligned(16))) uint32_t tab[TAB_ENTRIES * C];
  __shared__ uint32_t etab[128];
  __shared__ uint32_t wsum[NT / PLK_WAVE];
  __shared__ uint32_t wbad[NT / PLK_WAVE];
  TableFill<NT, C> fill;
  fill.load();
  uint32_t ev = 0;
  if (EXPLDS && threadIdx.x < PLK_GROUP_ORDER) ev = reinterpret_cast<const uint32_t*>(c_exp)[threadIdx.x];
  const uint64_t g = (uint64_t)blockIdx.x * NT + threadIdx.x;
  const uint32_t lane4 = (threadIdx.x & (C - 1u)) << 2;
  bool bad = false;
  uint32_t acc;
  if (HALF) {   // 8 points per thread: lanes 2t, 2t+1 split group t
    const uint64_t gr = g >> 1, h = g & 1;
    const uint2* pp = reinterpret_cast<const uint2*>(pts + 48 * gr + 24 * h);
    uint2 a0, a1, a2, sv;
    asm volatile("" ::: "memory");
    a0 = pp[0];
    asm volatile("" ::: "memory");
    a1 = pp[1];
    asm volatile("" ::: "memory");
    a2 = pp[2];
    asm volatile("" ::: "memory");
    sv = *reinterpret_cast<const uint2*>(sc + 16 * gr + 8 * h);
    if (!(ABL & 8)) {
      fill.store(tab);
      if (EXPLDS && threadIdx.x < PLK_GROUP_ORDER) etab[threadIdx.x] = ev;
      __syncthreads();
    }
    const uint32_t w[12] = {a0.x, a0.y, a1.x, a1.y, a2.x, a2.y, 0, 0, 0, 0, 0, 0};
    uint32_t d[8];
    d[0] = dval<C, 0, ABL>(w, tab, lane4);   d[1] = dval<C, 1, ABL>(w, tab, lane4);
    d[2] = dval<C, 2, ABL>(w, tab, lane4);   d[3] = dval<C, 3, ABL>(w, tab, lane4);
    d[4] = dval<C, 4, ABL>(w, tab, lane4);   d[5] = dval<C, 5, ABL>(w, tab, lane4);
    d[6] = dval<C, 6, ABL>(w, tab, lane4);   d[7] = dval<C, 7, ABL>(w, tab, lane4);
    if (ABL & 2) {
#pragma unroll
      for (int j = 0; j < 8; j++) d[j] = w[j % 6] + j;
    }
    uint32_t o = 0;
#pragma unroll
    for (int j = 0; j < 8; j++) o |= d[j];
    bad = o >= 256u;
    const uint32_t sw[2] = {sv.x, sv.y};
    acc = 0;
#pragma unroll
    for (int j = 0; j < 2; j++) {
      const uint32_t packed = __builtin_amdgcn_perm(__builtin_amdgcn_perm(d[4 * j + 3], d[4 * j + 2], 0x0C0C0400u),
                                                    __builtin_amdgcn_perm(d[4 * j + 1], d[4 * j], 0x0C0C0400u),
                                                    0x05040100u);
      acc = __builtin_amdgcn_udot4(packed, sw[j], acc, false);
    }
  } else {
  const uint4* p4 = reinterpret_cast<const uint4*>(pts);
  const uint4* s4 = reinterpret_cast<const uint4*>(sc);
  uint4 q0, q1, q2, s;
  asm volatile("" ::: "memory");
  if (ORDER == 1) {
    s = s4[g];
    asm volatile("" ::: "memory");
  }
  q0 = p4[3 * g];
  asm volatile("" ::: "memory");
  q1 = p4[3 * g + 1];
  asm volatile("" ::: "memory");
  q2 = p4[3 * g + 2];
  asm volatile("" ::: "memory");
  if (ORDER != 1) s = s4[g];
  fill.store(tab);
  if (EXPLDS && threadIdx.x < PLK_GROUP_ORDER) etab[threadIdx.x] = ev;
  __syncthreads();
  if (ORDER != 2) {
    Group gr{q0, q1, q2, s};
    acc = group_sum<C>(gr, tab, lane4, bad);
  } else {
    const uint32_t w[12] = {q0.x, q0.y, q0.z, q0.w, q1.x, q1.y, q1.z, q1.w, q2.x, q2.y, q2.z, q2.w};
    uint32_t d[16];
    d[0] = dval<C, 0>(w, tab, lane4);   d[1] = dval<C, 1>(w, tab, lane4);
    d[2] = dval<C, 2>(w, tab, lane4);   d[3] = dval<C, 3>(w, tab, lane4);
    d[4] = dval<C, 4>(w, tab, lane4);   d[5] = dval<C, 5>(w, tab, lane4);
    d[6] = dval<C, 6>(w, tab, lane4);   d[7] = dval<C, 7>(w, tab, lane4);
    d[8] = dval<C, 8>(w, tab, lane4);   d[9] = dval<C, 9>(w, tab, lane4);
    d[10] = dval<C, 10>(w, tab, lane4); d[11] = dval<C, 11>(w, tab, lane4);
    d[12] = dval<C, 12>(w, tab, lane4); d[13] = dval<C, 13>(w, tab, lane4);
    d[14] = dval<C, 14>(w, tab, lane4); d[15] = dval<C, 15>(w, tab, lane4);
    uint32_t o = 0;
#pragma unroll
    for (int j = 0; j < 16; j++) o |= d[j];
    bad = o >= 256u;
    const uint32_t sw[4] = {s.x, s.y, s.z, s.w};
    acc = 0;
#pragma unroll
    for (int j = 0; j < 4; j++) {
      const uint32_t packed = __builtin_amdgcn_perm(__builtin_amdgcn_perm(d[4 * j + 3], d[4 * j + 2], 0x0C0C0400u),
                                                    __builtin_amdgcn_perm(d[4 * j + 1], d[4 * j], 0x0C0C0400u),
                                                    0x05040100u);
      acc = __builtin_amdgcn_udot4(packed, sw[j], acc, false);
    }
  }
  }
  acc %= PLK_GROUP_ORDER;
  const uint32_t wave = threadIdx.x / PLK_WAVE;
  const uint32_t ws = plk_wave_sum(acc);
  const uint64_t anybad = __ballot(bad);
  if ((threadIdx.x & (PLK_WAVE - 1)) == 0) {
    wsum[wave] = ws;
    wbad[wave] = anybad != 0;
  }
  __syncthreads();
  if (threadIdx.x != 0) return;
  uint32_t bs = 0, bb_ = 0;
#pragma unroll
  for (int k = 0; k < NT / PLK_WAVE; k++) {
    bs += wsum[k];
    bb_ |= wbad[k];
  }
  const uint32_t X = gridDim.x;
  if (ABL & 4) {   // no finish: plain store of the block partial
    res->pad[blockIdx.x % 11] = bs + bb_;
    return;
  }
  if (ABL & 16) {  // non-returning add into the block's shard word only
    atomicAdd(shw + 16 * (blockIdx.x % SH), (unsigned long long)bs);
    return;
  }
  unsigned long long add =
      (unsigned long long)(bs % PLK_GROUP_ORDER) | (1ull << 32) | ((unsigned long long)(bb_ != 0) << 48);
  const uint32_t early = X > (uint32_t)LATE ? X - LATE : 0u;   // blocks >= early add straight into top
  if (blockIdx.x < early) {
    const uint32_t sh = blockIdx.x % SH;
    const uint32_t in_shard = (early - sh + SH - 1) / SH;
    unsigned long long* word = shw + 16 * sh;
    const unsigned long long old = atomicAdd(word, add);
    if (((old >> 32) & 0xFFFFull) != in_shard - 1) return;
    const unsigned long long tot = old + add;
    atomicExch(word, 0ull);
    if (ABL & 32) {   // one level: the shard's last block stores the shard total
      res->pad[sh % 11] = (uint32_t)tot;
      return;
    }
    add = (unsigned long long)((uint32_t)(tot & 0xFFFFFFFFull) % PLK_GROUP_ORDER) | (1ull << 32) |
          ((unsigned long long)((tot >> 48) != 0) << 48);
  }
  const uint32_t arrivals = (early < SH ? early : SH) + (X - early);
  const unsigned long long old = atomicAdd(&res->top, add);
  if (((old >> 32) & 0xFFFFull) != arrivals - 1) return;
  const unsigned long long tot = old + add;
  const uint32_t lg = (uint32_t)(tot & 0xFFFFFFFFull) % PLK_GROUP_ORDER;
  res->log = lg;
  res->irregular = (uint32_t)(tot >> 48);
  if (EXPLDS) {
    *reinterpret_cast<uint32_t*>(res->g1) = etab[lg] & 0xFFFFFFu;
  } else {
    res->g1[0] = c_exp[4 * lg + 0];
    res->g1[1] = c_exp[4 * lg + 1];
    res->g1[2] = c_exp[4 * lg + 2];
    res->g1[3] = 0;
  }
  atomicExch(&res->top, 0ull);
}

}  // namespace lab2
using namespace lab2;

int main(int argc, char** argv) {
  const int reps = argc > 1 ? atoi(argv[1]) : 200;
  const int rounds = argc > 2 ? atoi(argv[2]) : 1;
  const uint64_t n = 1ull << 22, ng = n >> 4;
  const int sets = 40;
  uint8_t *pts, *sc;
  CK(hipMalloc(&pts, 3 * n * sets));
  CK(hipMalloc(&sc, n * sets));
  {
    std::vector<uint8_t> h(4 * n);
    uint64_t x = 88172645463325252ull;
    for (auto& b : h) {
      x ^= x << 13; x ^= x >> 7; x ^= x << 17;
      b = (uint8_t)(x >> 24);
    }
    for (int s = 0; s < sets; s++) {
      CK(hipMemcpy(pts + 3 * n * s, h.data(), 3 * n, hipMemcpyHostToDevice));
      CK(hipMemcpy(sc + n * s, h.data() + 3 * n, n, hipMemcpyHostToDevice));
    }
  }
  uint32_t ytab[512];
  for (int i = 0; i < 512; i++) ytab[i] = (uint32_t)((i & 0xFF) ^ 1) << 16 | (uint32_t)(i % 102);
  uint8_t e4[408] = {0}, inv[101] = {0};
  if (plk_msm_upload_tables(ytab, e4, inv)) return 1;
  PlkMsmResult* lres;
  CK(hipMalloc(&lres, sizeof(PlkMsmResult) * 2));
  CK(hipMemset(lres, 0, sizeof(PlkMsmResult) * 2));
  unsigned long long* shw;
  CK(hipMalloc(&shw, 64 * 128));
  CK(hipMemset(shw, 0, 64 * 128));
  hipStream_t st;
  CK(hipStreamCreate(&st));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  struct V { std::string name; std::function<void(int)> f; };
  std::vector<V> vs;
#define VARX(NT, C, ORD, EL, SH, HF)                                                                    \
  vs.push_back({"v<" #NT "," #C ",ord" #ORD "," #EL ",sh" #SH ",half" #HF ">", [=](int s) {             \
                  hipLaunchKernelGGL((k_v<NT, C, ORD, EL, SH, HF>), dim3((uint32_t)(ng * (HF ? 2 : 1) / NT)), \
                                     dim3(NT), 0, st, pts + 3 * n * s, sc + n * s, lres, shw);          \
                }})
#define VAR(NT, C, ORD, EL) VARX(NT, C, ORD, EL, 8, false)
#define VARL(SH, LATE)                                                                                \
  vs.push_back({"half_sh" #SH "_late" #LATE, [=](int s) {                                              \
                  hipLaunchKernelGGL((k_v<512, 1, 2, true, SH, true, 0, LATE>), dim3((uint32_t)(ng * 2 / 512)), \
                                     dim3(512), 0, st, pts + 3 * n * s, sc + n * s, lres, shw);        \
                }})
#define VARA(ABL)                                                                                     \
  vs.push_back({"half_sh32_abl" #ABL, [=](int s) {                                                     \
                  hipLaunchKernelGGL((k_v<512, 1, 2, true, 32, true, ABL>), dim3((uint32_t)(ng * 2 / 512)), \
                                     dim3(512), 0, st, pts + 3 * n * s, sc + n * s, lres, shw);        \
                }})
#define LIBG(NT, G, C, BL)                                                                          \
  vs.push_back({"lib<" #NT "," #G "," #C "> grid " #BL, [=](int s) {                                \
                  hipLaunchKernelGGL((msm_dlog_kernel<true, NT, G, C, false>), dim3(BL, 1), dim3(NT), 0, st, \
                                     pts + 3 * n * s, 3 * n, sc + n * s, n, n,                       \
                                     (uint32_t)((n >> 4) / ((uint64_t)BL * NT * G)), lres + 1);      \
                }})
  LIBG(512, 1, 1, 512);
  VARA(0);    // full (half groups, 32 shards)
  VARA(32);   // one level of returning atomics
  VARA(4);    // no finish
  VARL(32, 8);
  VARL(32, 16);
  VARL(32, 32);
  VARL(16, 16);
  VARL(32, 64);
  for (int round = 0; round < rounds; round++)
    for (const V& v : vs) {
      for (int w = 0; w < 3; w++) v.f(w);
      CK(hipEventRecord(a, st));
      for (int r = 0; r < reps; r++) v.f(r % sets);
      CK(hipEventRecord(b, st));
      CK(hipEventSynchronize(b));
      CK(hipGetLastError());
      float ms;
      CK(hipEventElapsedTime(&ms, a, b));
      printf("%-28s %7.2f us/launch (events, back to back)\n", v.name.c_str(), ms * 1e3 / reps);
      fflush(stdout);
    }
  return 0;
}
