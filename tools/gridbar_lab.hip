// Grid-barrier lab (tuning aid, not part of the product): what does a kernel boundary cost a
// two-pass transform of 2^20 u32 (4 MiB), next to a device-wide barrier inside one launch?
//   two    : pass 1 (block b: a 256-row x 16-column tile, rows 4096 words apart -- the high pass
//            of a 2^20 NTT) in place, then pass 2 (block b: the contiguous words [4096 b, +4096))
//            as two launches
//   fused  : the same two passes in ONE launch of one block per CU, separated by a hierarchical
//            grid barrier (per-XCD arrival words, then one top word every block polls)
//   flat   : the same with one arrival word for all blocks
// The data is touched (x = x * 3 + 1) so the passes cannot be elided; timing is what matters.
// Every poll loop is bounded (a block that is never resident cannot hang the launch).
//
//   hipcc -O3 --offload-arch=gfx950 -std=c++17 tools/gridbar_lab.hip -o tools/gridbar_lab
//   rocprofv3 --kernel-trace --stats -d out -o run -- ./tools/gridbar_lab
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

constexpr int NT = 1024, E = 4, TILE = NT * E;   // 4096 words per tile
constexpr int K = 20;                            // 2^20 words

struct Bar {
  unsigned long long xcd[8][16];   // one 128-byte line per XCD
  unsigned long long top[16];
  unsigned long long flat[16];
  unsigned int err[32];
};

// WT: pass 1 stores write through to the device coherence point (agent-scope relaxed atomic
// stores) and pass 2 loads bypass the XCD's L2 (agent-scope relaxed atomic loads), so the
// barrier needs no L2 writeback / invalidate fences
template <bool WT = false>
__device__ __forceinline__ void pass1(uint32_t* d, uint32_t b) {
  // tile b: columns [16 b', +16) of the 256 rows (row stride 4096 words), b' = b mod 256
  const uint32_t c = threadIdx.x & 15, r0 = threadIdx.x >> 4;
  uint32_t v[E];
#pragma unroll
  for (int k = 0; k < E; k++) v[k] = d[(size_t)(r0 + 64 * k) * 4096 + (b & 255) * 16 + c];
#pragma unroll
  for (int k = 0; k < E; k++) v[k] = v[k] * 3u + 1u;
#pragma unroll
  for (int k = 0; k < E; k++) {
    uint32_t* q = d + (size_t)(r0 + 64 * k) * 4096 + (b & 255) * 16 + c;
    if (WT) __hip_atomic_store(q, v[k], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    else *q = v[k];
  }
}
template <bool WT = false>
__device__ __forceinline__ void pass2(uint32_t* d, uint32_t b) {
  uint32_t v[E];
#pragma unroll
  for (int k = 0; k < E; k++) {
    uint32_t* q = d + (size_t)b * TILE + k * NT + threadIdx.x;
    v[k] = WT ? __hip_atomic_load(q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : *q;
  }
#pragma unroll
  for (int k = 0; k < E; k++) v[k] = v[k] * 5u + 7u;
#pragma unroll
  for (int k = 0; k < E; k++) d[(size_t)b * TILE + k * NT + threadIdx.x] = v[k];
}

__device__ __forceinline__ bool poll_ge(unsigned long long* w, unsigned long long target) {
  for (int i = 0; i < (1 << 20); i++) {
    if (__hip_atomic_load(w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= target) return true;
    __builtin_amdgcn_s_sleep(1);
  }
  return false;
}

// barrier number `gen` (1, 2, ...) over all launches so far: the host passes the launch epoch
template <bool HIER, bool FENCE = true>
__device__ __forceinline__ void grid_barrier(Bar* bar, unsigned long long gen) {
  if (!FENCE) __builtin_amdgcn_s_waitcnt(0);   // this thread's write-through stores have landed
  __syncthreads();
  if (threadIdx.x == 0) {
    if (FENCE) __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    bool ok;
    if (HIER) {
      const uint32_t s = blockIdx.x & 7, per = gridDim.x / 8;
      const unsigned long long old = atomicAdd(&bar->xcd[s][0], 1ull);
      if (old + 1 == gen * per) atomicAdd(&bar->top[0], 1ull);
      ok = poll_ge(&bar->top[0], gen * 8);
    } else {
      atomicAdd(&bar->flat[0], 1ull);
      ok = poll_ge(&bar->flat[0], gen * gridDim.x);
    }
    if (!ok) atomicOr(&bar->err[0], 1u);
    if (FENCE) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  }
  __syncthreads();
}

__global__ __launch_bounds__(NT) void k_pass1(uint32_t* d) { pass1(d, blockIdx.x); }
__global__ __launch_bounds__(NT) void k_pass2(uint32_t* d) { pass2(d, blockIdx.x); }
template <bool HIER>
__global__ __launch_bounds__(NT) void k_fused(uint32_t* d, Bar* bar, unsigned long long gen) {
  pass1(d, blockIdx.x);
  grid_barrier<HIER>(bar, gen);
  pass2(d, blockIdx.x);
}
__global__ __launch_bounds__(NT) void k_fused_wt(uint32_t* d, Bar* bar, unsigned long long gen) {
  pass1<true>(d, blockIdx.x);
  grid_barrier<true, false>(bar, gen);
  pass2<true>(d, blockIdx.x);
}
__global__ __launch_bounds__(NT) void k_bar_only(uint32_t* d, Bar* bar, unsigned long long gen) {
  grid_barrier<true, false>(bar, gen);
}
__global__ void k_empty() {}

int main() {
  const size_t words = 1ull << K;
  const int nbuf = 16;   // 64 MiB: Infinity-Cache resident, like a transform of freshly written data
  uint32_t* base;
  CK(hipMalloc(&base, words * 4 * nbuf));
  CK(hipMemset(base, 1, words * 4 * nbuf));
  Bar* bar;
  CK(hipMalloc(&bar, sizeof(Bar)));
  CK(hipMemset(bar, 0, sizeof(Bar)));
  int cus = 0;
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  const int blocks = (int)(words / TILE);   // 256
  printf("CUs %d, blocks %d\n", cus, blocks);
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  setvbuf(stdout, nullptr, _IONBF, 0);
  // the hierarchical modes share the xcd/top words, so they share one barrier count
  unsigned long long gen_h = 0, gen_f = 0;
  unsigned long long& gen_w = gen_h;
  unsigned long long& gen_b = gen_h;
  const int reps = 200;
  const char* names[] = {"two", "fused", "flat", "empty", "fused_wt", "bar_only"};
  // correctness of each data mode: one step on a fresh buffer vs the host
  {
    uint32_t* h = (uint32_t*)malloc(words * 4);
    for (int mode : {0, 1, 2, 4}) {
      for (size_t i = 0; i < words; i++) h[i] = (uint32_t)(i * 2654435761u);
      CK(hipMemcpy(base, h, words * 4, hipMemcpyHostToDevice));
      if (mode == 0) {
        hipLaunchKernelGGL(k_pass1, dim3(blocks), dim3(NT), 0, 0, base);
        hipLaunchKernelGGL(k_pass2, dim3(blocks), dim3(NT), 0, 0, base);
      } else if (mode == 1) hipLaunchKernelGGL(k_fused<true>, dim3(blocks), dim3(NT), 0, 0, base, bar, ++gen_h);
      else if (mode == 2) hipLaunchKernelGGL(k_fused<false>, dim3(blocks), dim3(NT), 0, 0, base, bar, ++gen_f);
      else hipLaunchKernelGGL(k_fused_wt, dim3(blocks), dim3(NT), 0, 0, base, bar, ++gen_w);
      CK(hipDeviceSynchronize());
      uint32_t* g = (uint32_t*)malloc(words * 4);
      CK(hipMemcpy(g, base, words * 4, hipMemcpyDeviceToHost));
      size_t bad = 0;
      for (size_t i = 0; i < words; i++) bad += g[i] != (((uint32_t)(i * 2654435761u) * 3u + 1u) * 5u + 7u);
      printf("check %-8s wrong words %zu\n", names[mode], bad);
      free(g);
    }
    free(h);
  }
  for (int mode = 0; mode < 6; mode++) {
    for (int warm = 0; warm < 2; warm++) {
      CK(hipDeviceSynchronize());
      CK(hipEventRecord(a));
      for (int r = 0; r < reps; r++) {
        uint32_t* d = base + (size_t)(r % nbuf) * words;
        if (mode == 0) {
          hipLaunchKernelGGL(k_pass1, dim3(blocks), dim3(NT), 0, 0, d);
          hipLaunchKernelGGL(k_pass2, dim3(blocks), dim3(NT), 0, 0, d);
        } else if (mode == 1) {
          hipLaunchKernelGGL(k_fused<true>, dim3(blocks), dim3(NT), 0, 0, d, bar, ++gen_h);
        } else if (mode == 2) {
          hipLaunchKernelGGL(k_fused<false>, dim3(blocks), dim3(NT), 0, 0, d, bar, ++gen_f);
        } else if (mode == 3) {
          hipLaunchKernelGGL(k_empty, dim3(blocks), dim3(NT), 0, 0);
        } else if (mode == 4) {
          hipLaunchKernelGGL(k_fused_wt, dim3(blocks), dim3(NT), 0, 0, d, bar, ++gen_w);
        } else {
          hipLaunchKernelGGL(k_bar_only, dim3(blocks), dim3(NT), 0, 0, d, bar, ++gen_b);
        }
      }
      CK(hipEventRecord(b));
      CK(hipEventSynchronize(b));
      CK(hipGetLastError());
      float ms;
      CK(hipEventElapsedTime(&ms, a, b));
      if (warm) printf("%-8s %.2f us per transform-shaped step\n", names[mode], ms * 1e3 / reps);
    }
  }
  unsigned err = 0;
  CK(hipMemcpy(&err, bar->err, 4, hipMemcpyDeviceToHost));
  printf("barrier timeouts: %u\n", err);
  return 0;
}
