// MSM load-layout lab (tuning aid, not part of the product).  Compares, at the bench's
// shape (B MSMs of 2^22 points per launch), the production msm_dlog_kernel with a variant
// whose loads are wave-coalesced: per 1024-point chunk a wave issues 4 x dwordx3 of points
// (768 contiguous bytes each) + 4 x dword of scalars (256 contiguous bytes each), lane l
// owning points 256 i + 4 l + t, instead of every lane reading its own 48 + 16 bytes
// (3 x dwordx4 at a 48-byte lane stride + 1 x dwordx4).  MODE 1/2: the two address patterns
// with the compute replaced by an xor (pure read rate).
//
//   hipcc -O3 --offload-arch=gfx950 tools/msm_layout_lab.hip -o tools/msm_layout_lab
#include "../plonk.c_amd/csrc/msm.hip"

#include <stdarg.h>
#include <stdio.h>

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

namespace {
struct W3 {
  uint32_t a, b, c;
};

template <int J>
__device__ __forceinline__ uint32_t pb3(const uint32_t (&w)[3]) {
  constexpr int o = 3 * J, d = o >> 2, b = o & 3;
  constexpr int d1 = (b + 2 <= 3) ? d : d + 1;
  constexpr uint32_t sel = 0x0Cu | ((uint32_t)b << 8) | ((uint32_t)(b + 1) << 16) | ((uint32_t)(b + 2) << 24);
  return __builtin_amdgcn_perm(w[d1], w[d], sel);
}

struct Chunk {
  W3 q[4];
  uint32_t s[4];
};

// MODE 0/1: wave-coalesced addresses; MODE 2: per-lane 48 B + 16 B (production pattern)
template <int MODE>
__device__ __forceinline__ Chunk load_chunk(const uint8_t* pts, const uint8_t* sc, uint64_t c, uint32_t lane) {
  Chunk r;
  if (MODE == 2) {
    const uint4* p4 = reinterpret_cast<const uint4*>(pts) + 3 * (c * 64 + lane);
    const uint4 a = p4[0], b = p4[1], d = p4[2];
    const uint4 s = reinterpret_cast<const uint4*>(sc)[c * 64 + lane];
    r.q[0] = W3{a.x, a.y, a.z};
    r.q[1] = W3{a.w, b.x, b.y};
    r.q[2] = W3{b.z, b.w, d.x};
    r.q[3] = W3{d.y, d.z, d.w};
    r.s[0] = s.x; r.s[1] = s.y; r.s[2] = s.z; r.s[3] = s.w;
  } else {
    const W3* p = reinterpret_cast<const W3*>(pts + c * 3072 + 12 * lane);
    const uint32_t* s = reinterpret_cast<const uint32_t*>(sc + c * 1024 + 4 * lane);
#pragma unroll
    for (int i = 0; i < 4; i++) r.q[i] = p[64 * i];
#pragma unroll
    for (int i = 0; i < 4; i++) r.s[i] = s[64 * i];
  }
  return r;
}

template <int MODE>
__device__ __forceinline__ uint32_t chunk_sum(const Chunk& ch, const uint32_t* tab, uint32_t lane4, bool& bad) {
  if (MODE != 0) {
    uint32_t x = 0;
#pragma unroll
    for (int i = 0; i < 4; i++) x ^= ch.q[i].a + ch.q[i].b + ch.q[i].c + ch.s[i];
    bad |= x == 0x12345u;
    return x & 63;
  }
  uint32_t part = 0;
#pragma unroll
  for (int i = 0; i < 4; i++) {
    const uint32_t w[3] = {ch.q[i].a, ch.q[i].b, ch.q[i].c};
    part += point_term(pb3<0>(w), ch.s[i] & 0xFFu, tab, lane4, bad);
    part += point_term(pb3<1>(w), (ch.s[i] >> 8) & 0xFFu, tab, lane4, bad);
    part += point_term(pb3<2>(w), (ch.s[i] >> 16) & 0xFFu, tab, lane4, bad);
    part += point_term(pb3<3>(w), ch.s[i] >> 24, tab, lane4, bad);
  }
  return part;
}
}  // namespace

template <int NT, int G, int MODE>
__global__ __launch_bounds__(NT) void wavec_kernel(const uint8_t* pts_base, uint64_t pstride, const uint8_t* sc_base,
                                                   uint64_t sstride, uint64_t n, PlkMsmResult* res_base) {
  __shared__ __attribute__((aligned(16))) uint32_t tab[TAB_ENTRIES * COPIES];
  __shared__ uint32_t wsum[NT / PLK_WAVE];
  const uint8_t* pts = pts_base + (uint64_t)blockIdx.y * pstride;
  const uint8_t* sc = sc_base + (uint64_t)blockIdx.y * sstride;
  PlkMsmResult* res = res_base + blockIdx.y;
  const uint32_t lane = threadIdx.x & 63u, wave = threadIdx.x >> 6;
  const uint32_t lane4 = (threadIdx.x & 31u) << 2;
  TableFill<NT> fill;
  fill.load();
  fill.store(tab);
  __syncthreads();
  const uint64_t W = (uint64_t)gridDim.x * (NT / 64);
  const uint64_t wg = (uint64_t)blockIdx.x * (NT / 64) + wave;
  const uint64_t nch = n >> 10;
  const uint32_t cnt = wg < nch ? (uint32_t)((nch - wg + W - 1) / W) : 0u;
  uint32_t acc = 0;
  bool bad = false;
  uint64_t c = wg;
  uint32_t k = 0;
  for (; k + G <= cnt; k += G) {
    Chunk cur[G];
    asm volatile("" ::: "memory");
#pragma unroll
    for (int j = 0; j < G; j++) {
      cur[j] = load_chunk<MODE>(pts, sc, c + j * W, lane);
      asm volatile("" ::: "memory");
    }
#pragma unroll
    for (int j = 0; j < G; j++) acc += chunk_sum<MODE>(cur[j], tab, lane4, bad) % PLK_GROUP_ORDER;
    c += G * W;
  }
  for (; k < cnt; k++) {
    const Chunk ch = load_chunk<MODE>(pts, sc, c, lane);
    acc += chunk_sum<MODE>(ch, tab, lane4, bad) % PLK_GROUP_ORDER;
    c += W;
  }
  if (blockIdx.x == 0)
    for (uint64_t i = (nch << 10) + threadIdx.x; i < n; i += NT)
      acc += point_term(encode(pts[3 * i], pts[3 * i + 1], pts[3 * i + 2]), sc[i], tab, lane4, bad);
  acc %= PLK_GROUP_ORDER;
  const uint32_t s = wave_sum(acc);
  if (lane == 0) wsum[wave] = s + (__ballot(bad) != 0 ? 1000u : 0u);
  __syncthreads();
  if (threadIdx.x != 0) return;
  uint32_t bs = 0;
  for (int w = 0; w < NT / PLK_WAVE; w++) bs += wsum[w];
  atomicAdd(reinterpret_cast<unsigned long long*>(&res->shard[blockIdx.x % PLK_MSM_SHARDS][0]),
            (unsigned long long)(bs % PLK_GROUP_ORDER) | (1ull << 32));
}

template <int NT, int G, int MODE>
static float time_wavec(int blocks_per_msm, int B, int L, uint8_t* pts, uint8_t* sc, uint64_t n, int sets,
                        PlkMsmResult* res, hipStream_t st, hipEvent_t a, hipEvent_t b) {
  float best = 1e30f;
  for (int rep = 0; rep < 3; rep++) {
    CK(hipEventRecord(a, st));
    for (int l = 0; l < L; l++) {
      const int s0 = (l * B) % sets;
      const int s = s0 + B > sets ? 0 : s0;
      hipLaunchKernelGGL((wavec_kernel<NT, G, MODE>), dim3(blocks_per_msm, B), dim3(NT), 0, st, pts + 3 * n * s,
                         3 * n, sc + n * s, n, n, res);
    }
    CK(hipEventRecord(b, st));
    CK(hipEventSynchronize(b));
    float ms;
    CK(hipEventElapsedTime(&ms, a, b));
    best = ms / L < best ? ms / L : best;
  }
  return best;
}

int main(int argc, char** argv) {
  const int log2n = argc > 1 ? atoi(argv[1]) : 22;
  const uint64_t n = 1ull << log2n;
  const int sets = 80;
  uint8_t *pts, *sc;
  CK(hipMalloc(&pts, 3 * n * sets));
  CK(hipMalloc(&sc, n * sets));
  CK(hipMemset(pts, 7, 3 * n * sets));
  CK(hipMemset(sc, 3, n * sets));
  PlkMsmResult* res;
  CK(hipMalloc(&res, 1 << 20));
  CK(hipMemset(res, 0, 1 << 20));
  hipStream_t st;
  CK(hipStreamCreate(&st));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  const int B = 40, L = 8;
  const double bytes = 4.0 * n * B;
  auto rep = [&](const char* name, float ms) {
    printf("%-34s %8.2f us/launch  %6.0f GB/s\n", name, ms * 1e3, bytes / (ms * 1e-3) / 1e9);
  };
  {
    float best = 1e30f;
    for (int r = 0; r < 3; r++) {
      CK(hipEventRecord(a, st));
      for (int l = 0; l < L; l++) {
        const int s0 = (l * B) % sets;
        const int s = s0 + B > sets ? 0 : s0;
        if (plk_msm_batch_launch(pts + 3 * n * s, 3 * n, sc + n * s, n, n, B, res, st) != PLK_OK) return 1;
      }
      CK(hipEventRecord(b, st));
      CK(hipEventSynchronize(b));
      float ms;
      CK(hipEventElapsedTime(&ms, a, b));
      best = ms / L < best ? ms / L : best;
    }
    rep("production msm_dlog", best);
  }
  CK(hipMemset(res, 0, 1 << 20));
  // production kernel, blocks per MSM swept (dynamic balance by oversubscription)
  const int shapes[][2] = {{40, 8}, {32, 8}, {24, 10}, {16, 16}, {12, 20}, {8, 20}, {4, 40}};
  for (auto& sh : shapes) {
    const int Bs = sh[0], Ls = sh[1];
    const double by = 4.0 * n * Bs;
    const int xs[] = {512 / Bs, 32, 64, 128, 192, 256, 384};
    for (int xi = 0; xi < 7; xi++) {
      const int x = xs[xi];
      for (int t = 0; t < 2; t++) {
        float best = 1e30f;
        for (int r = 0; r < 3; r++) {
          CK(hipEventRecord(a, st));
          for (int l = 0; l < Ls; l++) {
            const int s0 = (l * Bs) % sets;
            const int s = s0 + Bs > sets ? 0 : s0;
            if (t == 0)
              hipLaunchKernelGGL((msm_dlog_kernel<true, 512, 2>), dim3(x, Bs), dim3(512), 0, st, pts + 3 * n * s, 3 * n,
                                 sc + n * s, n, n, res);
            else
              hipLaunchKernelGGL((msm_dlog_kernel<true, 512, 1>), dim3(x, Bs), dim3(512), 0, st, pts + 3 * n * s, 3 * n,
                                 sc + n * s, n, n, res);
          }
          CK(hipEventRecord(b, st));
          CK(hipEventSynchronize(b));
          float ms;
          CK(hipEventElapsedTime(&ms, a, b));
          best = ms / Ls < best ? ms / Ls : best;
        }
        printf("B=%-2d G=%d blocks/msm=%-5d total=%-6d %8.2f us/launch  %6.0f GB/s\n", Bs, t ? 1 : 2, x, x * Bs,
               best * 1e3, by / (best * 1e-3) / 1e9);
      }
    }
  }
  return 0;
}
