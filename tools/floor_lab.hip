// Data-movement floor lab (tuning aid, not part of the product).  Round 2's
// gridbar_lab measured the two-pass 2^20 read-touch-write at ONE 4096-element tile per CU (256-row x
// 16-column high-pass tiles, 4096-word contiguous lo-pass tiles, 1024 threads): 8.5 us as two
// launches.  This measures the same data movement at other splits and block shapes -- more, smaller
// tiles per CU (2-4 blocks, 16-32 waves per CU), 2^11 x 2^9 and 2^10 x 2^10 splits, 16 / 32 / 64 B
// column segments, one word or 16 B per lane -- so that the single-transform floor is known at more
// than one configuration.  Every pass loads its tile, touches it (x = x * 3 + 1 / x * 5 + 7) and
// stores it in place; no butterflies, no exchanges.  Tiles are placed XCD-aware as in the engine
// (consecutive tiles on one XCD, so the column segments of one 128-byte line meet in one L2).
//
//   hipcc -O3 --offload-arch=gfx950 -std=c++17 tools/floor_lab.hip -o tools/floor_lab
//   ./tools/floor_lab [reps]     (rocprofv3 --pmc ... -- ./tools/floor_lab 8 for counters per kernel shape)
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#define CK(x)                                                         \
  do {                                                                \
    hipError_t e = (x);                                               \
    if (e != hipSuccess) {                                            \
      printf("%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e)); \
      exit(1);                                                        \
    }                                                                 \
  } while (0)

constexpr int K = 20;   // 2^20 words per transform

__device__ __forceinline__ uint32_t xcd_tile() {
  const uint32_t nb = gridDim.x, b = blockIdx.x;
  return (nb % 8 == 0) ? (b % 8) * (nb / 8) + b / 8 : b;
}

// high pass: a tile is 2^M rows x C columns (row stride 2^(K-M) words); a lane holds V consecutive
// columns of one row (V = 4: one 16-byte load), the block's lanes cover C / V column groups x rows
template <int M, int C, int NT, int V>
__global__ __launch_bounds__(NT) void k_hi(uint32_t* d) {
  constexpr int TILE = (1 << M) * C, E = TILE / NT / V, G = C / V, RSTEP = NT / G;
  static_assert(E >= 1 && NT % G == 0, "shape");
  constexpr uint32_t RS = 1u << (K - M);
  const uint32_t t = xcd_tile(), c = (threadIdx.x % G) * V, r0 = threadIdx.x / G;
  if constexpr (V == 4) {
    uint4 v[E];
#pragma unroll
    for (int k = 0; k < E; k++) v[k] = *(const uint4*)(d + (size_t)(r0 + RSTEP * k) * RS + t * C + c);
#pragma unroll
    for (int k = 0; k < E; k++) {
      v[k].x = v[k].x * 3u + 1u; v[k].y = v[k].y * 3u + 1u; v[k].z = v[k].z * 3u + 1u; v[k].w = v[k].w * 3u + 1u;
    }
#pragma unroll
    for (int k = 0; k < E; k++) *(uint4*)(d + (size_t)(r0 + RSTEP * k) * RS + t * C + c) = v[k];
  } else {
    uint32_t v[E];
#pragma unroll
    for (int k = 0; k < E; k++) v[k] = d[(size_t)(r0 + RSTEP * k) * RS + t * C + c];
#pragma unroll
    for (int k = 0; k < E; k++) v[k] = v[k] * 3u + 1u;
#pragma unroll
    for (int k = 0; k < E; k++) d[(size_t)(r0 + RSTEP * k) * RS + t * C + c] = v[k];
  }
}

// lo pass: contiguous tiles of 2^L words; a lane holds V consecutive words per load
template <int L, int NT, int V>
__global__ __launch_bounds__(NT) void k_lo(uint32_t* d) {
  constexpr int E = (1 << L) / NT / V;
  static_assert(E >= 1, "shape");
  uint32_t* q = d + ((size_t)xcd_tile() << L);
  if constexpr (V == 4) {
    uint4 v[E];
#pragma unroll
    for (int k = 0; k < E; k++) v[k] = ((const uint4*)q)[k * NT + threadIdx.x];
#pragma unroll
    for (int k = 0; k < E; k++) {
      v[k].x = v[k].x * 5u + 7u; v[k].y = v[k].y * 5u + 7u; v[k].z = v[k].z * 5u + 7u; v[k].w = v[k].w * 5u + 7u;
    }
#pragma unroll
    for (int k = 0; k < E; k++) ((uint4*)q)[k * NT + threadIdx.x] = v[k];
  } else {
    uint32_t v[E];
#pragma unroll
    for (int k = 0; k < E; k++) v[k] = q[k * NT + threadIdx.x];
#pragma unroll
    for (int k = 0; k < E; k++) v[k] = v[k] * 5u + 7u;
#pragma unroll
    for (int k = 0; k < E; k++) q[k * NT + threadIdx.x] = v[k];
  }
}

__global__ void k_empty() {}

struct Cfg {
  const char* name;
  void (*hi)(uint32_t*);
  int hi_blocks, hi_nt;
  void (*lo)(uint32_t*);
  int lo_blocks, lo_nt;
};

#define HI(M, C, NT, V) (void (*)(uint32_t*))k_hi<M, C, NT, V>, (1 << (K - M)) / (C), NT
#define LO(L, NT, V) (void (*)(uint32_t*))k_lo<L, NT, V>, 1 << (K - (L)), NT

int main(int argc, char** argv) {
  const size_t words = 1ull << K;
  const int nbuf = 16;   // 64 MiB: Infinity-Cache resident, like a transform of freshly written data
  uint32_t* base;
  CK(hipMalloc(&base, words * 4 * nbuf));
  CK(hipMemset(base, 1, words * 4 * nbuf));
  int cus = 0;
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  printf("# floor_lab: two-pass 2^20 u32 read-touch-write (no butterflies), %d CUs, 16 rotating buffers\n", cus);
  printf("# name: high pass M rows-bits x C cols (blocks x threads), lo pass 2^L words (blocks x threads), V words/lane\n");
  const Cfg cfgs[] = {
      {"r02 M8xC16/1024 | L12/1024 | V1", HI(8, 16, 1024, 1), LO(12, 1024, 1)},
      {"M8xC16/1024 | L12/1024 | V4", HI(8, 16, 1024, 4), LO(12, 1024, 4)},
      {"M8xC16/512 | L12/512 | V1", HI(8, 16, 512, 1), LO(12, 512, 1)},
      {"M8xC8/512 | L12/1024 | V1", HI(8, 8, 512, 1), LO(12, 1024, 1)},
      {"M9xC4/512 | L11/512 | V1", HI(9, 4, 512, 1), LO(11, 512, 1)},
      {"M9xC4/512 | L11/512 | V4", HI(9, 4, 512, 4), LO(11, 512, 4)},
      {"M9xC4/256 | L11/256 | V1", HI(9, 4, 256, 1), LO(11, 256, 1)},
      {"M9xC4/256 | L11/256 | V4", HI(9, 4, 256, 4), LO(11, 256, 4)},
      {"M9xC8/1024 | L11/512 | V1", HI(9, 8, 1024, 1), LO(11, 512, 1)},
      {"M9xC8/512 | L11/512 | V4", HI(9, 8, 512, 4), LO(11, 512, 4)},
      {"M10xC4/1024 | L10/256 | V1", HI(10, 4, 1024, 1), LO(10, 256, 1)},
      {"M10xC4/512 | L10/256 | V4", HI(10, 4, 512, 4), LO(10, 256, 4)},
      {"M10xC2/512 | L10/256 | V1", HI(10, 2, 512, 1), LO(10, 256, 1)},
      {"M10xC4/256 | L10/128 | V4", HI(10, 4, 256, 4), LO(10, 128, 4)},
  };
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  setvbuf(stdout, nullptr, _IONBF, 0);
  const int reps = argc > 1 ? atoi(argv[1]) : 400;   // (a few for --pmc runs: every dispatch is counted)
  // correctness of the indexing: every word touched exactly once per pass
  {
    uint32_t* h = (uint32_t*)malloc(words * 4);
    uint32_t* g = (uint32_t*)malloc(words * 4);
    for (const Cfg& c : cfgs) {
      for (size_t i = 0; i < words; i++) h[i] = (uint32_t)(i * 2654435761u);
      CK(hipMemcpy(base, h, words * 4, hipMemcpyHostToDevice));
      hipLaunchKernelGGL(c.hi, dim3(c.hi_blocks), dim3(c.hi_nt), 0, 0, base);
      hipLaunchKernelGGL(c.lo, dim3(c.lo_blocks), dim3(c.lo_nt), 0, 0, base);
      CK(hipDeviceSynchronize());
      CK(hipMemcpy(g, base, words * 4, hipMemcpyDeviceToHost));
      size_t bad = 0;
      for (size_t i = 0; i < words; i++) bad += g[i] != (((uint32_t)(i * 2654435761u) * 3u + 1u) * 5u + 7u);
      if (bad) printf("CHECK FAILED %s: %zu wrong words\n", c.name, bad);
    }
    free(h);
    free(g);
  }
  for (const Cfg& c : cfgs) {
    float best[3] = {1e9f, 1e9f, 1e9f};
    for (int part = 0; part < 3; part++) {   // 0: both passes, 1: high only, 2: lo only
      for (int trial = 0; trial < 3; trial++) {
        CK(hipDeviceSynchronize());
        CK(hipEventRecord(a));
        for (int r = 0; r < reps; r++) {
          uint32_t* d = base + (size_t)(r % nbuf) * words;
          if (part != 2) hipLaunchKernelGGL(c.hi, dim3(c.hi_blocks), dim3(c.hi_nt), 0, 0, d);
          if (part != 1) hipLaunchKernelGGL(c.lo, dim3(c.lo_blocks), dim3(c.lo_nt), 0, 0, d);
        }
        CK(hipEventRecord(b));
        CK(hipEventSynchronize(b));
        CK(hipGetLastError());
        float ms;
        CK(hipEventElapsedTime(&ms, a, b));
        if (trial && ms * 1e3f / reps < best[part]) best[part] = ms * 1e3f / reps;
      }
    }
    printf("%-34s hi %4d x %4d  lo %4d x %4d   two-pass %6.2f us   hi alone %5.2f   lo alone %5.2f\n", c.name,
           c.hi_blocks, c.hi_nt, c.lo_blocks, c.lo_nt, best[0], best[1], best[2]);
  }
  for (int nb : {256, 512, 1024}) {
    float best = 1e9f;
    for (int trial = 0; trial < 3; trial++) {
      CK(hipEventRecord(a));
      for (int r = 0; r < reps; r++) hipLaunchKernelGGL(k_empty, dim3(nb), dim3(256), 0, 0);
      CK(hipEventRecord(b));
      CK(hipEventSynchronize(b));
      float ms;
      CK(hipEventElapsedTime(&ms, a, b));
      if (trial && ms * 1e3f / reps < best) best = ms * 1e3f / reps;
    }
    printf("empty launch, %4d blocks: %.2f us\n", nb, best);
  }
  return 0;
}
