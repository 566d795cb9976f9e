// SWAR probe (tuning aid, not part of the product): the round-1 numdiv variant that summed the
// numerator lincomb two bytes per 16-bit lane reported its bytes-2/3 lanes as zero on the device
// while a CPU emulation was exact (tuning log).  The variant was not kept; this
// probe restates that arithmetic in the forms it could have taken and compares the device with
// the host bit for bit, printing the first mismatch.  The ISA of each form is in the
// --save-temps output (v_mul_u32_u24 / v_mad_u32_u16 / v_pk_* selection is what to look at).
//
//   hipcc -O3 --offload-arch=gfx950 -std=c++17 tools/swar_probe.hip -o tools/swar_probe
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#define CK(x)                                                         \
  do {                                                                \
    hipError_t e = (x);                                               \
    if (e != hipSuccess) {                                            \
      printf("%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e)); \
      return 1;                                                       \
    }                                                                 \
  } while (0)

constexpr int NT = 6;   // lincomb terms (the numerator of t(x) with its sum group)

// form 0: per-byte accumulators (the kept form)
// form 1: two 16-bit lanes per accumulator: lo = bytes 0, 2; hi = bytes 1, 3
// form 2: form 1 with the coefficient as a uint8 (zero-extended byte load)
// form 3: form 1 through 16-bit vector types (packed v_pk_mad_u16)
__host__ __device__ inline void lincomb(int form, const uint32_t* w, const uint8_t* cf, uint8_t out[4]) {
  if (form == 0) {
    uint32_t a[4] = {0, 0, 0, 0};
    for (int t = 0; t < NT; t++)
      for (int b = 0; b < 4; b++) a[b] += cf[t] * ((w[t] >> (8 * b)) & 0xFFu);
    for (int b = 0; b < 4; b++) out[b] = (uint8_t)(a[b] % 17u);
    return;
  }
  uint32_t lo = 0, hi = 0;
  for (int t = 0; t < NT; t++) {
    const uint32_t c = form == 2 ? (uint32_t)(uint8_t)cf[t] : (uint32_t)cf[t];
    lo += c * (w[t] & 0x00FF00FFu);
    hi += c * ((w[t] >> 8) & 0x00FF00FFu);
  }
  out[0] = (uint8_t)((lo & 0xFFFFu) % 17u);
  out[1] = (uint8_t)((hi & 0xFFFFu) % 17u);
  out[2] = (uint8_t)((lo >> 16) % 17u);
  out[3] = (uint8_t)((hi >> 16) % 17u);
}

__device__ inline void lincomb_pk(const uint32_t* w, const uint8_t* cf, uint8_t out[4]) {
  typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));
  u16x2 lo = {0, 0}, hi = {0, 0};
  for (int t = 0; t < NT; t++) {
    const u16x2 c = {(unsigned short)cf[t], (unsigned short)cf[t]};
    const u16x2 l = {(unsigned short)(w[t] & 0xFFu), (unsigned short)((w[t] >> 16) & 0xFFu)};
    const u16x2 h = {(unsigned short)((w[t] >> 8) & 0xFFu), (unsigned short)((w[t] >> 24) & 0xFFu)};
    lo += c * l;
    hi += c * h;
  }
  out[0] = (uint8_t)(lo.x % 17u);
  out[1] = (uint8_t)(hi.x % 17u);
  out[2] = (uint8_t)(lo.y % 17u);
  out[3] = (uint8_t)(hi.y % 17u);
}

__global__ void probe(int form, const uint32_t* words, const uint8_t* cfs, uint8_t* out, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint32_t w[NT];
  uint8_t cf[NT];
  for (int t = 0; t < NT; t++) {
    w[t] = words[(size_t)i * NT + t];
    cf[t] = cfs[(size_t)i * NT + t];
  }
  if (form == 3) lincomb_pk(w, cf, out + 4 * (size_t)i);
  else lincomb(form, w, cf, out + 4 * (size_t)i);
}

// form 4, in a kernel of its own (adding it to probe() changes how the forms above compile):
// form 1 with the masked words made opaque to the instruction combiner
__global__ void probe_opaque(const uint32_t* words, const uint8_t* cfs, uint8_t* out, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint32_t lo = 0, hi = 0;
  for (int t = 0; t < NT; t++) {
    const uint32_t w = words[(size_t)i * NT + t];
    uint32_t ml = w & 0x00FF00FFu, mh = (w >> 8) & 0x00FF00FFu;
    asm volatile("" : "+v"(ml), "+v"(mh));
    const uint32_t c = cfs[(size_t)i * NT + t];
    lo += c * ml;
    hi += c * mh;
  }
  out[4 * (size_t)i + 0] = (uint8_t)((lo & 0xFFFFu) % 17u);
  out[4 * (size_t)i + 1] = (uint8_t)((hi & 0xFFFFu) % 17u);
  out[4 * (size_t)i + 2] = (uint8_t)((lo >> 16) % 17u);
  out[4 * (size_t)i + 3] = (uint8_t)((hi >> 16) % 17u);
}

int main() {
  const int n = 1 << 20;
  uint32_t* hw = (uint32_t*)malloc(sizeof(uint32_t) * n * NT);
  uint8_t* hc = (uint8_t*)malloc(n * NT);
  uint8_t* ho = (uint8_t*)malloc(4 * (size_t)n);
  uint64_t s = 0x9E3779B97F4A7C15ull;
  for (size_t i = 0; i < (size_t)n * NT; i++) {
    s ^= s << 13; s ^= s >> 7; s ^= s << 17;
    // canonical bytes (< 17) in every byte lane, coefficients < 17: every lane sum < 2^16
    hw[i] = (uint32_t)(s % 17) | (uint32_t)((s >> 8) % 17) << 8 | (uint32_t)((s >> 16) % 17) << 16 |
            (uint32_t)((s >> 24) % 17) << 24;
    hc[i] = (uint8_t)((s >> 40) % 17);
  }
  uint32_t* dw;
  uint8_t *dc, *dout;
  CK(hipMalloc(&dw, sizeof(uint32_t) * n * NT));
  CK(hipMalloc(&dc, n * NT));
  CK(hipMalloc(&dout, 4 * (size_t)n));
  CK(hipMemcpy(dw, hw, sizeof(uint32_t) * n * NT, hipMemcpyHostToDevice));
  CK(hipMemcpy(dc, hc, n * NT, hipMemcpyHostToDevice));
  int bad_total = 0;
  for (int form = 0; form < 5; form++) {
    CK(hipMemset(dout, 0xAB, 4 * (size_t)n));
    if (form == 4) hipLaunchKernelGGL(probe_opaque, dim3(n / 256), dim3(256), 0, 0, dw, dc, dout, n);
    else hipLaunchKernelGGL(probe, dim3(n / 256), dim3(256), 0, 0, form, dw, dc, dout, n);
    CK(hipGetLastError());
    CK(hipMemcpy(ho, dout, 4 * (size_t)n, hipMemcpyDeviceToHost));
    int bad = 0;
    for (int i = 0; i < n; i++) {
      uint8_t want[4];
      lincomb(0, hw + (size_t)i * NT, hc + (size_t)i * NT, want);
      for (int b = 0; b < 4; b++)
        if (ho[4 * (size_t)i + b] != want[b]) {
          if (bad < 3) printf("form %d: item %d byte %d: device %u host %u\n", form, i, b, ho[4 * (size_t)i + b], want[b]);
          bad++;
        }
    }
    printf("form %d: %d mismatching bytes of %d\n", form, bad, 4 * n);
    bad_total += bad;
  }
  return bad_total ? 2 : 0;
}
