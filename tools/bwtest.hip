// HBM read-pattern microbenchmark (tuning aid, not part of the product).
//   contig : lane i reads 16 B at base + 16 i (+ grid stride)         -- ideal stream
//   msm    : thread t reads 48 B at 48 t (3 x dwordx4) + 16 B at 16 t  -- the MSM layout
// Each launch reads `bytes` from one of several buffers (> 512 MiB total, Infinity-Cache
// cold).  Prints GB/s from hipEvents around single launches.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s\n", hipGetErrorString(e)); exit(1); } } while (0)

__global__ __launch_bounds__(1024) void contig(const uint4* __restrict__ p, size_t n16, unsigned* out) {
  unsigned acc = 0;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n16; i += (size_t)gridDim.x * blockDim.x) {
    uint4 v = p[i];
    acc ^= v.x + v.y + v.z + v.w;
  }
  if (acc == 0x12345678u) out[0] = acc;
}

__global__ __launch_bounds__(1024) void msm_like(const uint4* __restrict__ p, const uint4* __restrict__ s,
                                                 size_t ngroups, unsigned* out) {
  unsigned acc = 0;
  for (size_t g = blockIdx.x * (size_t)blockDim.x + threadIdx.x; g < ngroups; g += (size_t)gridDim.x * blockDim.x) {
    uint4 a = p[3 * g], b = p[3 * g + 1], c = p[3 * g + 2], d = s[g];
    acc ^= a.x + b.y + c.z + d.w + a.w + b.x + c.y + d.z;
  }
  if (acc == 0x12345678u) out[0] = acc;
}

int main(int argc, char** argv) {
  const size_t bytes = argc > 1 ? strtoull(argv[1], 0, 0) : (16u << 20);  // per launch
  const int nbuf = (int)((700ull << 20) / bytes) + 1;
  char* base;
  CK(hipMalloc(&base, bytes * nbuf));
  CK(hipMemset(base, 1, bytes * nbuf));
  unsigned* out;
  CK(hipMalloc(&out, 64));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  const int threads[] = {256, 1024};
  for (int mode = 0; mode < 2; mode++)
    for (int ti = 0; ti < 2; ti++)
      for (int blocks : {256, 512, 1024, 2048, 4096}) {
        const int th = threads[ti];
        float best = 1e9, sum = 0;
        const int reps = 40;
        for (int r = 0; r < reps; r++) {
          const char* buf = base + (size_t)(r % nbuf) * bytes;
          CK(hipEventRecord(a));
          if (mode == 0)
            hipLaunchKernelGGL(contig, dim3(blocks), dim3(th), 0, 0, (const uint4*)buf, bytes / 16, out);
          else
            hipLaunchKernelGGL(msm_like, dim3(blocks), dim3(th), 0, 0, (const uint4*)buf,
                               (const uint4*)(buf + bytes / 4 * 3), bytes / 64, out);
          CK(hipEventRecord(b));
          CK(hipEventSynchronize(b));
          float ms;
          CK(hipEventElapsedTime(&ms, a, b));
          if (r >= 5) { best = ms < best ? ms : best; sum += ms; }
        }
        const float avg = sum / (reps - 5);
        printf("%-8s bytes=%zu threads=%4d blocks=%5d  avg %.2f us (%.0f GB/s)  best %.2f us (%.0f GB/s)\n",
               mode ? "msm" : "contig", bytes, th, blocks, avg * 1e3, bytes / (avg * 1e-3) / 1e9, best * 1e3,
               bytes / (best * 1e-3) / 1e9);
      }
  // empty-kernel event overhead
  float sum = 0;
  for (int r = 0; r < 50; r++) {
    CK(hipEventRecord(a));
    hipLaunchKernelGGL(contig, dim3(1), dim3(64), 0, 0, (const uint4*)base, 0, out);
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms;
    CK(hipEventElapsedTime(&ms, a, b));
    sum += ms;
  }
  printf("empty kernel (event pair) avg %.2f us\n", sum / 50 * 1e3);
  return 0;
}
