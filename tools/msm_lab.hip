// MSM kernel lab (tuning aid, not part of the product): times msm_dlog_kernel launch shapes
// on synthetic data, next to a plain streaming read of the same bytes.  Built several times
// with -DPLK_MSM_DIAG=0..3 (see msm.hip) to split the fixed per-launch cost into table,
// finish and streaming parts.  Geometry comes from the PLK_MSM_* environment variables.
//
//   hipcc -O3 --offload-arch=gfx950 -DPLK_MSM_DIAG=1 tools/msm_lab.hip -o tools/msm_lab_d1
//   ./tools/msm_lab_d1 [log2n=22]
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

#define CK(x)                                                      \
  do {                                                             \
    hipError_t e = (x);                                            \
    if (e != hipSuccess) {                                         \
      printf("%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e)); \
      exit(1);                                                     \
    }                                                              \
  } while (0)

__global__ __launch_bounds__(1024) void lab_contig(const uint4* __restrict__ p, size_t np16, const uint4* __restrict__ s,
                                                   size_t ns16, unsigned* out) {
  unsigned acc = 0;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < np16 + ns16; i += (size_t)gridDim.x * blockDim.x) {
    uint4 v = i < np16 ? p[i] : s[i - np16];
    acc ^= v.x + v.y + v.z + v.w;
  }
  if (acc == 0x12345678u) out[0] = acc;
}

int main(int argc, char** argv) {
  const int log2n = argc > 1 ? atoi(argv[1]) : 22;
  const uint64_t n = 1ull << log2n;
  const int sets = 40;
  uint8_t *pts, *sc;
  CK(hipMalloc(&pts, 3 * n * sets));
  CK(hipMalloc(&sc, n * sets));
  CK(hipMemset(pts, 7, 3 * n * sets));
  CK(hipMemset(sc, 3, n * sets));
  PlkMsmResult* res;
  CK(hipMalloc(&res, 1 << 20));
  CK(hipMemset(res, 0, 1 << 20));
  unsigned* out;
  CK(hipMalloc(&out, 64));
  hipStream_t st;
  CK(hipStreamCreate(&st));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  const int batches[] = {1, 8, 40};
  for (int bi = 0; bi < 3; bi++) {
    const int B = batches[bi];
    const int L = B == 40 ? 8 : (B == 8 ? 20 : 80);
    int th, bl, g;
    plk_msm_geometry(n, B, &th, &bl, &g, nullptr, nullptr);
    float best = 1e30f;
    for (int rep = 0; rep < 3; rep++) {
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
    const double bytes = 4.0 * n * B;
    printf("diag=%d B=%-3d threads=%-4d blocks=%-4d G=%d  %8.2f us/launch  %6.0f GB/s\n", PLK_MSM_DIAG, B, th, bl, g,
           best * 1e3, bytes / (best * 1e-3) / 1e9);
    // the same bytes as a plain streaming read (16 B per lane, 256 x 1024 threads)
    float bestc = 1e30f;
    for (int rep = 0; rep < 3; rep++) {
      CK(hipEventRecord(a, st));
      for (int l = 0; l < L; l++) {
        const int s0 = (l * B) % sets;
        const int s = s0 + B > sets ? 0 : s0;
        hipLaunchKernelGGL(lab_contig, dim3(256), dim3(1024), 0, st, (const uint4*)(pts + 3 * n * s),
                           (size_t)(3 * n * B / 16), (const uint4*)(sc + n * s), (size_t)(n * B / 16), out);
      }
      CK(hipEventRecord(b, st));
      CK(hipEventSynchronize(b));
      float ms;
      CK(hipEventElapsedTime(&ms, a, b));
      bestc = ms / L < bestc ? ms / L : bestc;
    }
    if (PLK_MSM_DIAG == 0)
      printf("        contig read of the same bytes (1 launch)              %8.2f us/launch  %6.0f GB/s\n",
             bestc * 1e3, bytes / (bestc * 1e-3) / 1e9);
  }
  return 0;
}
