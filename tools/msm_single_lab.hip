// Single-MSM lab (tuning aid, not part of the product): where does the fixed cost of ONE
// 2^22-point MSM launch go?  Times, under rocprofv3 --kernel-trace, variants of the one-pass
// discrete-log kernel (msm.hip) that differ in launch shape, LDS table copies and the
// cross-block finish, next to a bare streaming read and an empty kernel of the same grid.
// Inputs rotate over 40 sets (640 MiB > the 256 MiB Infinity Cache): every launch reads cold.
//
//   hipcc -O3 --offload-arch=gfx950 -std=c++17 tools/msm_single_lab.hip -o tools/msm_single_lab
//   rocprofv3 --kernel-trace --stats -d out -o run -- ./tools/msm_single_lab
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

#define CK(x)                                                           \
  do {                                                                  \
    hipError_t e = (x);                                                 \
    if (e != hipSuccess) {                                              \
      printf("%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e));   \
      exit(1);                                                          \
    }                                                                   \
  } while (0)

namespace lab {
__constant__ uint32_t c_tab[512];

struct Rec {
  unsigned long long top;
  uint32_t log, irregular;
  uint8_t g1[4];
  uint32_t pad[27];
  unsigned long long shard[32][16];
};

template <int J>
__device__ __forceinline__ uint32_t point_bytes(const uint32_t (&w)[12]) {
  constexpr int o = 3 * J, d = o >> 2, b = o & 3;
  constexpr int d1 = (b + 2 <= 3) ? d : d + 1;
  constexpr uint32_t sel = 0x0Cu | ((uint32_t)b << 8) | ((uint32_t)(b + 1) << 16) | ((uint32_t)(b + 2) << 24);
  return __builtin_amdgcn_perm(w[d1], w[d], sel);
}

template <int COPIES, int J>
__device__ __forceinline__ void term(const uint32_t (&w)[12], const uint32_t (&sw)[4], const uint32_t* tab,
                                     uint32_t lane4, bool& bad, uint32_t& part) {
  constexpr int SH = COPIES == 1 ? 2 : (COPIES == 2 ? 3 : (COPIES == 4 ? 4 : 5));
  const uint32_t k = point_bytes<J>(w);
  const uint32_t idx = (k >> 16) & 0x1FFu;
  const uint32_t e = *reinterpret_cast<const uint32_t*>(reinterpret_cast<const char*>(tab) + ((idx << SH) | lane4));
  const uint32_t d = e - k;
  bad |= d >= 256u;
  part += (d & 0xFFu) * ((sw[J >> 2] >> (8 * (J & 3))) & 0xFFu);
}

template <int COPIES>
__device__ __forceinline__ uint32_t gsum(uint4 q0, uint4 q1, uint4 q2, uint4 s, const uint32_t* tab, uint32_t lane4,
                                         bool& bad) {
  const uint32_t w[12] = {q0.x, q0.y, q0.z, q0.w, q1.x, q1.y, q1.z, q1.w, q2.x, q2.y, q2.z, q2.w};
  const uint32_t sw[4] = {s.x, s.y, s.z, s.w};
  uint32_t p = 0;
  term<COPIES, 0>(w, sw, tab, lane4, bad, p);  term<COPIES, 1>(w, sw, tab, lane4, bad, p);
  term<COPIES, 2>(w, sw, tab, lane4, bad, p);  term<COPIES, 3>(w, sw, tab, lane4, bad, p);
  term<COPIES, 4>(w, sw, tab, lane4, bad, p);  term<COPIES, 5>(w, sw, tab, lane4, bad, p);
  term<COPIES, 6>(w, sw, tab, lane4, bad, p);  term<COPIES, 7>(w, sw, tab, lane4, bad, p);
  term<COPIES, 8>(w, sw, tab, lane4, bad, p);  term<COPIES, 9>(w, sw, tab, lane4, bad, p);
  term<COPIES, 10>(w, sw, tab, lane4, bad, p); term<COPIES, 11>(w, sw, tab, lane4, bad, p);
  term<COPIES, 12>(w, sw, tab, lane4, bad, p); term<COPIES, 13>(w, sw, tab, lane4, bad, p);
  term<COPIES, 14>(w, sw, tab, lane4, bad, p); term<COPIES, 15>(w, sw, tab, lane4, bad, p);
  return p;
}

// FIN 0: plain store of the block partial (no finish; lower bound)
// FIN 1: two-level ticketed atomics over SH shard words (the library's form at SH = 8)
// FIN 2: one level, SH shard words, no ticket: non-returning adds (lower bound of the atomics alone)
template <int NT, int COPIES, int FIN, int SH>
__global__ __launch_bounds__(NT) void k_msm(const uint8_t* pts, const uint8_t* sc, uint64_t n, Rec* res) {
  __shared__ __attribute__((aligned(16))) uint32_t tab[512 * COPIES];
  __shared__ uint32_t wsum[NT / 64], wbad[NT / 64];
  const uint4* p4 = reinterpret_cast<const uint4*>(pts);
  const uint4* s4 = reinterpret_cast<const uint4*>(sc);
  const uint64_t ng = n >> 4;
  const uint64_t stride = (uint64_t)gridDim.x * NT;
  uint64_t g = (uint64_t)blockIdx.x * NT + threadIdx.x;
  constexpr int PER = 512 * COPIES / NT > 0 ? 512 * COPIES / NT : 1;
  uint32_t tv[PER];
#pragma unroll
  for (int j = 0; j < PER; j++) tv[j] = c_tab[((threadIdx.x + j * NT) / COPIES) & 511];
  const uint32_t lane4 = (threadIdx.x & (COPIES - 1u)) << 2;
  uint32_t acc = 0;
  bool bad = false;
  bool first = true;
  for (; g < ng; g += stride) {
    asm volatile("" ::: "memory");
    const uint4 q0 = p4[3 * g], q1 = p4[3 * g + 1], q2 = p4[3 * g + 2], s = s4[g];
    asm volatile("" ::: "memory");
    if (first) {
#pragma unroll
      for (int j = 0; j < PER; j++)
        if (threadIdx.x + j * NT < 512 * COPIES) tab[threadIdx.x + j * NT] = tv[j];
      __syncthreads();
      first = false;
    }
    acc += gsum<COPIES>(q0, q1, q2, s, tab, lane4, bad) % 102u;
  }
  acc %= 102u;
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) acc += __shfl_xor(acc, off, 64);
  const uint64_t anyb = __ballot(bad);
  if ((threadIdx.x & 63) == 0) {
    wsum[threadIdx.x / 64] = acc;
    wbad[threadIdx.x / 64] = anyb != 0;
  }
  __syncthreads();
  if (threadIdx.x != 0) return;
  uint32_t bs = 0, bb = 0;
#pragma unroll
  for (int k = 0; k < NT / 64; k++) { bs += wsum[k]; bb |= wbad[k]; }
  unsigned long long add = (unsigned long long)(bs % 102u) | (1ull << 32) | ((unsigned long long)(bb != 0) << 48);
  if (FIN == 0) {
    res->pad[blockIdx.x % 11] = (uint32_t)add;
    return;
  }
  const uint32_t X = gridDim.x;
  const uint32_t sh = blockIdx.x % SH;
  unsigned long long* word = &res->shard[sh][0];
  if (FIN == 2) {
    atomicAdd(word, add);
    return;
  }
  const uint32_t in_shard = (X - sh + SH - 1) / SH;
  const unsigned long long old = atomicAdd(word, add);
  if (((old >> 32) & 0xFFFFull) != in_shard - 1) return;
  const unsigned long long tot = old + add;
  atomicExch(word, 0ull);
  if (FIN == 3) {
    res->pad[sh] = (uint32_t)(tot & 0xFFFFFFFFull) % 102u | (uint32_t)((tot >> 48) != 0) << 31;
    return;
  }
  add = (unsigned long long)((uint32_t)(tot & 0xFFFFFFFFull) % 102u) | (1ull << 32) |
        ((unsigned long long)((tot >> 48) != 0) << 48);
  const uint32_t arrivals = X < SH ? X : SH;
  const unsigned long long o2 = atomicAdd(&res->top, add);
  if (((o2 >> 32) & 0xFFFFull) != arrivals - 1) return;
  const unsigned long long t2 = o2 + add;
  res->log = (uint32_t)(t2 & 0xFFFFFFFFull) % 102u;
  res->irregular = (uint32_t)(t2 >> 48);
  atomicExch(&res->top, 0ull);
}

// Cost ladder, one group of 16 points per thread, table in C copies:
//   ST 0: bare read (xor of the loaded words, no LDS)
//   ST 1: + table load, LDS fill and barrier (words still xor-ed, no lookups)
//   ST 2: + the 16 lookups per group (the real partial), per-thread store if it is a magic value
//   ST 3: + block reduction (wave sums, LDS, barrier), thread 0 stores the partial
//   ST 4: + non-returning 64-bit atomic of the partial into one of 8 shard words
//   ST 5: + returning atomic, the shard's last block stores the shard total (one level)
//   ST 6: + the shard's last block adds into the top word, the last shard writes the result (library)
template <int NT, int C, int ST, int G = 1>
__global__ __launch_bounds__(NT) void k_ladder(const uint8_t* pts, const uint8_t* sc, uint64_t n, Rec* res) {
  __shared__ __attribute__((aligned(16))) uint32_t tab[512 * C];
  __shared__ uint32_t wsum[NT / 64], wbad[NT / 64];
  const uint4* p4 = reinterpret_cast<const uint4*>(pts);
  const uint4* s4 = reinterpret_cast<const uint4*>(sc);
  const uint64_t stride = (uint64_t)gridDim.x * NT;
  const uint64_t g0 = (uint64_t)blockIdx.x * NT + threadIdx.x;   // grid x G covers n / 16 exactly
  uint32_t tv = 0;
  if (ST >= 1) tv = c_tab[(threadIdx.x / C) & 511];
  uint4 q[G][4];
  asm volatile("" ::: "memory");
#pragma unroll
  for (int j = 0; j < G; j++) {
    const uint64_t g = g0 + j * stride;
    q[j][0] = p4[3 * g]; q[j][1] = p4[3 * g + 1]; q[j][2] = p4[3 * g + 2]; q[j][3] = s4[g];
    asm volatile("" ::: "memory");
  }
  if (ST >= 1) {
    if (threadIdx.x < 512 * C) tab[threadIdx.x] = tv;
    __syncthreads();
  }
  uint32_t acc = 0;
  bool bad = false;
#pragma unroll
  for (int j = 0; j < G; j++) {
    if (ST < 2) {
      acc += q[j][0].x + q[j][1].y + q[j][2].z + q[j][3].w + q[j][0].w + q[j][1].x + q[j][2].y + q[j][3].z +
             q[j][0].y + q[j][0].z + q[j][1].z + q[j][1].w + q[j][2].x + q[j][2].w + q[j][3].x + q[j][3].y;
    } else {
      acc += gsum<C>(q[j][0], q[j][1], q[j][2], q[j][3], tab, (threadIdx.x & (C - 1u)) << 2, bad) % 102u;
    }
  }
  if (ST <= 2) {
    if (acc == 0x12345678u || bad) res->pad[0] = acc;
    return;
  }
  acc = plk_wave_sum(acc);
  const uint64_t anyb = __ballot(bad);
  if ((threadIdx.x & 63) == 0) {
    wsum[threadIdx.x / 64] = acc;
    wbad[threadIdx.x / 64] = anyb != 0;
  }
  __syncthreads();
  if (threadIdx.x != 0) return;
  uint32_t bs = 0, bb = 0;
#pragma unroll
  for (int k = 0; k < NT / 64; k++) { bs += wsum[k]; bb |= wbad[k]; }
  unsigned long long add = (unsigned long long)(bs % 102u) | (1ull << 32) | ((unsigned long long)(bb != 0) << 48);
  if (ST == 3) {
    res->pad[blockIdx.x % 11] = (uint32_t)add;
    return;
  }
  const uint32_t X = gridDim.x, sh = blockIdx.x % 8u;
  unsigned long long* word = &res->shard[sh][0];
  if (ST == 4) {
    atomicAdd(word, add);
    return;
  }
  const uint32_t in_shard = (X - sh + 7) / 8;
  const unsigned long long old = atomicAdd(word, add);
  if (((old >> 32) & 0xFFFFull) != in_shard - 1) return;
  const unsigned long long tot = old + add;
  atomicExch(word, 0ull);
  if (ST == 5) {
    res->pad[sh] = (uint32_t)(tot & 0xFFFFFFFFull) % 102u;
    return;
  }
  add = (unsigned long long)((uint32_t)(tot & 0xFFFFFFFFull) % 102u) | (1ull << 32);
  const unsigned long long o2 = atomicAdd(&res->top, add);
  if (((o2 >> 32) & 0xFFFFull) != 7) return;
  res->log = (uint32_t)((o2 + add) & 0xFFFFFFFFull) % 102u;
  atomicExch(&res->top, 0ull);
}

template <int NT>
__global__ __launch_bounds__(NT) void k_read(const uint8_t* pts, const uint8_t* sc, uint64_t n, Rec* res) {
  const uint4* p4 = reinterpret_cast<const uint4*>(pts);
  const uint4* s4 = reinterpret_cast<const uint4*>(sc);
  const uint64_t ng = n >> 4;
  uint32_t acc = 0;
  for (uint64_t g = (uint64_t)blockIdx.x * NT + threadIdx.x; g < ng; g += (uint64_t)gridDim.x * NT) {
    const uint4 q0 = p4[3 * g], q1 = p4[3 * g + 1], q2 = p4[3 * g + 2], s = s4[g];
    acc ^= q0.x + q1.y + q2.z + s.w + q0.w + q1.x + q2.y + s.z;
  }
  if (acc == 0x12345678u) res->pad[0] = acc;
}

template <int NT, int G>
__global__ __launch_bounds__(NT) void k_readg(const uint8_t* pts, const uint8_t* sc, uint64_t n, Rec* res) {
  const uint4* p4 = reinterpret_cast<const uint4*>(pts);
  const uint4* s4 = reinterpret_cast<const uint4*>(sc);
  const uint64_t ng = n >> 4;
  const uint64_t stride = (uint64_t)gridDim.x * NT;
  uint32_t acc = 0;
  for (uint64_t g = (uint64_t)blockIdx.x * NT + threadIdx.x; g < ng; g += stride * G) {
    uint4 q[G][4];
#pragma unroll
    for (int j = 0; j < G; j++) {
      const uint64_t gj = g + j * stride < ng ? g + j * stride : ng - 1;
      q[j][0] = p4[3 * gj]; q[j][1] = p4[3 * gj + 1]; q[j][2] = p4[3 * gj + 2]; q[j][3] = s4[gj];
    }
#pragma unroll
    for (int j = 0; j < G; j++) acc ^= q[j][0].x + q[j][1].y + q[j][2].z + q[j][3].w + q[j][0].w + q[j][1].x;
  }
  if (acc == 0x12345678u) res->pad[0] = acc;
}

template <int NT>
__global__ __launch_bounds__(NT) void k_empty(const uint8_t*, const uint8_t*, uint64_t n, Rec* res) {
  if (n == 12345) res->pad[0] = 1;
}

}  // namespace lab
using namespace lab;

typedef void (*KFn)(const uint8_t*, const uint8_t*, uint64_t, Rec*);

int main(int argc, char** argv) {
  const int log2n = argc > 1 ? atoi(argv[1]) : 22;
  const int reps = argc > 2 ? atoi(argv[2]) : 100;
  const bool isolated = argc > 3 && atoi(argv[3]) != 0;   // synchronize after every launch
  const uint64_t n = 1ull << log2n;
  const int sets = 40;
  uint8_t *pts, *sc;
  CK(hipMalloc(&pts, 3 * n * sets));
  CK(hipMalloc(&sc, n * sets));
  CK(hipMemset(pts, 7, 3 * n * sets));
  CK(hipMemset(sc, 3, n * sets));
  uint32_t t[512];
  for (int i = 0; i < 512; i++) t[i] = (uint32_t)(i * 2654435761u);
  CK(hipMemcpyToSymbol(HIP_SYMBOL(c_tab), t, sizeof t));
  Rec* res;
  CK(hipMalloc(&res, sizeof(Rec) * 2));
  CK(hipMemset(res, 0, sizeof(Rec) * 2));
  hipStream_t st;
  CK(hipStreamCreate(&st));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  PlkMsmResult* lres;
  CK(hipMalloc(&lres, sizeof(PlkMsmResult) * 64));
  CK(hipMemset(lres, 0, sizeof(PlkMsmResult) * 64));
  uint32_t ytab[512];
  for (int i = 0; i < 512; i++) ytab[i] = (uint32_t)((i & 0xFF) ^ 1) << 16;
  uint8_t e4[408] = {0}, inv[101] = {0};
  if (plk_msm_upload_tables(ytab, e4, inv)) return 1;
  typedef std::function<void(int s)> L;
  struct V { std::string name; L f; int batch; };
  std::vector<V> vs;
  const uint64_t ng = n >> 4;
  auto raw = [&](const char* name, KFn f, int nt, int blocks) {
    vs.push_back({name, [=](int s) { hipLaunchKernelGGL(f, dim3(blocks), dim3(nt), 0, st, pts + 3 * n * s, sc + n * s, n, res); }, 1});
  };
#define LIB(NT, G, C, B)                                                                       \
  vs.push_back({"lib<" #NT "," #G "," #C "> x" #B, [=](int s) {                               \
                  int th, bl, g, c;                                                          \
                  plk_msm_geometry(n, B, &th, &bl, &g, &c, nullptr);                                 \
                  hipLaunchKernelGGL((msm_dlog_kernel<true, NT, G, C, false>), dim3(bl, B), dim3(NT), 0, st, \
                                     pts + 3 * n * s, 3 * n, sc + n * s, n, n,                \
                                     (uint32_t)((n >> 4) / ((uint64_t)bl * NT * G)), lres);   \
                }, B})
#define LIBG(NT, G, C, BL)                                                                     \
  vs.push_back({"lib<" #NT "," #G "," #C "> grid " #BL, [=](int s) {                         \
                  hipLaunchKernelGGL((msm_dlog_kernel<true, NT, G, C, false>), dim3(BL, 1), dim3(NT), 0, st, \
                                     pts + 3 * n * s, 3 * n, sc + n * s, n, n,                \
                                     (uint32_t)((n >> 4) / ((uint64_t)BL * NT * G)), lres);   \
                }, 1})
  const int set = argc > 5 ? atoi(argv[5]) : 0;
  if (set == 1) {   // geometry and cost-ladder exploration
    raw("empty_256x256", k_empty<256>, 256, 256);
    raw("empty_512x256", k_empty<512>, 512, 256);
    raw("empty_1024x256", k_empty<1024>, 1024, 256);
    raw("empty_512x512", k_empty<512>, 512, 512);
    raw("readg_256_g4_x256", k_readg<256, 4>, 256, (int)(ng / 1024));
    raw("readg_256_g8_x128", k_readg<256, 8>, 256, (int)(ng / 2048));
    raw("readg_512_g2_x256", k_readg<512, 2>, 512, (int)(ng / 1024));
    raw("readg_512_g4_x128", k_readg<512, 4>, 512, (int)(ng / 2048));
    raw("readg_1024_g1_x256", k_readg<1024, 1>, 1024, (int)(ng / 1024));
    raw("readg_512_g1_x512", k_readg<512, 1>, 512, (int)(ng / 512));
    raw("L0_512_c1", k_ladder<512, 1, 0, 1>, 512, (int)(ng / 512));
    raw("L1_512_c1", k_ladder<512, 1, 1, 1>, 512, (int)(ng / 512));
    raw("L2_512_c1", k_ladder<512, 1, 2, 1>, 512, (int)(ng / 512));
    raw("L3_512_c1", k_ladder<512, 1, 3, 1>, 512, (int)(ng / 512));
    raw("L4_512_c1", k_ladder<512, 1, 4, 1>, 512, (int)(ng / 512));
    raw("L5_512_c1", k_ladder<512, 1, 5, 1>, 512, (int)(ng / 512));
    raw("L6_512_c1", k_ladder<512, 1, 6, 1>, 512, (int)(ng / 512));
    raw("L0_256_g4_c1", k_ladder<256, 1, 0, 4>, 256, (int)(ng / 1024));
    raw("L1_256_g4_c1", k_ladder<256, 1, 1, 4>, 256, (int)(ng / 1024));
    raw("L2_256_g4_c1", k_ladder<256, 1, 2, 4>, 256, (int)(ng / 1024));
    raw("L3_256_g4_c1", k_ladder<256, 1, 3, 4>, 256, (int)(ng / 1024));
    raw("L6_256_g4_c1", k_ladder<256, 1, 6, 4>, 256, (int)(ng / 1024));
  }
  if (set == 0) {
  raw("empty_512x512", k_empty<512>, 512, (int)(ng / 512));
  raw("ladder0_read", k_ladder<512, 1, 0>, 512, (int)(ng / 512));
  raw("ladder6_g1_c8", k_ladder<512, 8, 6, 1>, 512, (int)(ng / 512));
  raw("ladder6_g2_c8", k_ladder<512, 8, 6, 2>, 512, (int)(ng / 1024));
  LIBG(512, 1, 8, 512);
  LIBG(512, 2, 8, 256);
  LIBG(512, 1, 1, 512);
  LIBG(256, 2, 8, 512);
  LIBG(1024, 1, 8, 256);
  LIB(512, 2, 8, 40);
  LIB(512, 2, 1, 40);
  }
  const int rounds = argc > 4 ? atoi(argv[4]) : 1;
  for (int round = 0; round < rounds; round++)
  for (const V& v : vs) {
    const int per = v.batch;
    const int R = per == 1 ? reps : (per == 8 ? reps / 4 : reps / 10);
    for (int w = 0; w < 3; w++) v.f(0);
    CK(hipEventRecord(a, st));
    for (int r = 0; r < R; r++) {
      const int s0 = (r * per) % sets;
      v.f(s0 + per > sets ? 0 : s0);
      if (isolated) CK(hipStreamSynchronize(st));
    }
    CK(hipEventRecord(b, st));
    CK(hipEventSynchronize(b));
    CK(hipGetLastError());
    float ms;
    CK(hipEventElapsedTime(&ms, a, b));
    printf("%-28s %7.2f us/launch (events, back to back)  %6.0f GB/s\n", v.name.c_str(), ms * 1e3 / R,
           4.0 * n * per / (ms * 1e-3 / R) / 1e9);
    fflush(stdout);
  }
  return 0;
}
