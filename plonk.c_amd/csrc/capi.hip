// C ABI of libplonkhip (include/plonkhip.h): context, device buffers, host-buffer wrappers
// around the gfx950 kernels in msm.hip and ntt.hip.
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <mutex>
#include <vector>

#include "plk_device.h"
#include "plk_internal.h"

namespace {

thread_local char g_err[512] = "";

struct Ctx {
  std::mutex mu;
  bool ready = false;
  int device = -1;
  hipStream_t st = nullptr;
  uint8_t gen[3] = {0, 0, 0};
  // MSM staging
  uint8_t* d_pts = nullptr;
  size_t cap_pts = 0;
  uint8_t* d_sc = nullptr;
  size_t cap_sc = 0;
  PlkMsmResult* d_res = nullptr;
  // poly_mul staging
  uint8_t* d_a = nullptr;
  size_t cap_a = 0;
  uint8_t* d_b = nullptr;
  size_t cap_b = 0;
  uint8_t* d_out = nullptr;
  size_t cap_out = 0;
  uint32_t* d_nz = nullptr;
  void* d_work = nullptr;
  size_t cap_work = 0;
} g;

// ---- E(F101) tables, built from the group law on canonical points ----------------------
struct HP { int x, y, inf; };

int md(int v) { v %= PLK_GF_P; return v < 0 ? v + PLK_GF_P : v; }
int inv101(int a) {  // a^99 mod 101 (Fermat, 0 -> 0), same as the reference gf_inv
  int r = 1, b = md(a), e = PLK_GF_P - 2;
  while (e) { if (e & 1) r = r * b % PLK_GF_P; b = b * b % PLK_GF_P; e >>= 1; }
  return r;
}
HP hp_add(HP a, HP b) {
  if (a.inf) return b;
  if (b.inf) return a;
  int m;
  if (a.x == b.x) {
    if (md(a.y + b.y) == 0) return HP{0, 0, 1};
    m = md(3 * a.x * a.x) * inv101(md(2 * a.y)) % PLK_GF_P;
  } else {
    m = md(b.y - a.y) * inv101(md(b.x - a.x)) % PLK_GF_P;
  }
  const int xr = md(m * m - a.x - b.x);
  const int yr = md(m * (a.x - xr) - a.y);
  return HP{xr, yr, 0};
}

int build_group_tables(uint8_t gen_out[3]) {
  std::vector<HP> pts;
  for (int x = 0; x < PLK_GF_P; x++)
    for (int y = 0; y < PLK_GF_P; y++)
      if (y * y % PLK_GF_P == (x * x * x + 3) % PLK_GF_P) pts.push_back(HP{x, y, 0});
  if (pts.size() + 1 != PLK_GROUP_ORDER) {
    plk_set_error("E(F101) has %zu points, expected 102", pts.size() + 1);
    return PLK_ERR_ARG;
  }
  HP g0{0, 0, 1};
  for (const HP& p : pts) {  // first (x, y) point of order 102
    HP q = p;
    int ord = 1;
    while (!q.inf && ord <= PLK_GROUP_ORDER) { q = hp_add(q, p); ord++; }
    if (ord == PLK_GROUP_ORDER) { g0 = p; break; }
  }
  if (g0.inf) {
    plk_set_error("no generator of order 102 found");
    return PLK_ERR_ARG;
  }
  static int logt[PLK_GF_P][PLK_GF_P];
  for (auto& row : logt)
    for (int& v : row) v = -1;
  uint8_t exp4[PLK_GROUP_ORDER * 4];
  HP q{0, 0, 1};
  for (int k = 0; k < PLK_GROUP_ORDER; k++) {
    exp4[4 * k + 0] = (uint8_t)q.x;
    exp4[4 * k + 1] = (uint8_t)q.y;
    exp4[4 * k + 2] = (uint8_t)q.inf;
    exp4[4 * k + 3] = 0;
    if (!q.inf) logt[q.x][q.y] = k;
    q = hp_add(q, g0);
  }
  // Lookup table of the MSM kernel (msm.hip): cubing is a bijection of GF(101), so each y
  // has exactly one x on the curve.  Index y | (inf & 1) << 8; a point encoded as
  // k = x << 8 | y << 16 | inf << 24 is canonical iff E[idx] - k < 256, and then that
  // difference is its log.  Entries that must never match get a wrong y byte.
  uint32_t ytab[512];
  for (int i = 0; i < 512; i++) ytab[i] = (uint32_t)((i & 0xFF) ^ 1) << 16;
  for (int x = 0; x < PLK_GF_P; x++)
    for (int y = 0; y < PLK_GF_P; y++)
      if (logt[x][y] >= 0) ytab[y] = (uint32_t)x << 8 | (uint32_t)y << 16 | (uint32_t)logt[x][y];
  ytab[256] = 1u << 24;  // identity {0, 0, 1}: log 0
  for (int y = 0; y < PLK_GF_P; y++)
    if ((ytab[y] >> 16 & 0xFF) != (uint32_t)y) {
      plk_set_error("E(F101): no point with y = %d", y);
      return PLK_ERR_ARG;
    }
  uint8_t inv[PLK_GF_P];
  for (int a = 0; a < PLK_GF_P; a++) inv[a] = (uint8_t)inv101(a);
  gen_out[0] = (uint8_t)g0.x;
  gen_out[1] = (uint8_t)g0.y;
  gen_out[2] = 0;
  return plk_msm_upload_tables(ytab, exp4, inv);
}

template <class T>
int grow(T** p, size_t* cap, size_t need) {
  if (*cap >= need && *p) return PLK_OK;
  size_t n = *cap ? *cap : 4096;
  while (n < need) n *= 2;
  if (*p) (void)hipFree(*p);
  *p = nullptr;
  *cap = 0;
  hipError_t e = hipMalloc((void**)p, n);
  if (e != hipSuccess) {
    plk_set_error("hipMalloc(%zu) failed: %s", n, hipGetErrorString(e));
    return PLK_ERR_NOMEM;
  }
  *cap = n;
  return PLK_OK;
}

int init_locked(int device) {
  if (g.ready) return PLK_OK;
  int count = 0;
  if (hipGetDeviceCount(&count) != hipSuccess || count <= 0) {
    plk_set_error("no HIP device available (libplonkhip has no CPU fallback)");
    return PLK_ERR_NODEV;
  }
  if (device < 0) {
    const char* e = getenv("PLK_DEVICE");
    device = e ? atoi(e) : 0;
  }
  if (device >= count) {
    plk_set_error("device %d out of range (%d devices)", device, count);
    return PLK_ERR_NODEV;
  }
  PLK_HIP(hipSetDevice(device));
  PLK_HIP(hipStreamCreateWithFlags(&g.st, hipStreamNonBlocking));
  int rc = build_group_tables(g.gen);
  if (rc) return rc;
  if ((rc = plk_ntt_init_tables())) return rc;
  PLK_HIP(hipMalloc((void**)&g.d_res, sizeof(PlkMsmResult)));
  PLK_HIP(hipMemset(g.d_res, 0, sizeof(PlkMsmResult)));
  PLK_HIP(hipMalloc((void**)&g.d_nz, 16));
  g.device = device;
  g.ready = true;
  return PLK_OK;
}

int ensure(void) {
  if (g.ready) return hipSetDevice(g.device) == hipSuccess ? PLK_OK : PLK_ERR_HIP;
  return init_locked(-1);
}

// Device entry points run on exactly the stream they are given; NULL is HIP's null stream
// (torch's default stream also has handle 0).  g.st is used only by the host-buffer calls.
hipStream_t pick(void* s) { return (hipStream_t)s; }

}  // namespace

void plk_set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof g_err, fmt, ap);
  va_end(ap);
}

extern "C" {

const char* plk_last_error(void) { return g_err; }
const char* plk_version(void) { return "libplonkhip 0.1 gfx950"; }

int plk_device_count(void) {
  int c = 0;
  if (hipGetDeviceCount(&c) != hipSuccess) return 0;
  return c;
}

int plk_init(int device) {
  std::lock_guard<std::mutex> lk(g.mu);
  return init_locked(device);
}

void plk_shutdown(void) {
  std::lock_guard<std::mutex> lk(g.mu);
  if (!g.ready) return;
  (void)hipStreamSynchronize(g.st);
  (void)hipFree(g.d_pts); (void)hipFree(g.d_sc); (void)hipFree(g.d_res);
  (void)hipFree(g.d_a); (void)hipFree(g.d_b); (void)hipFree(g.d_out); (void)hipFree(g.d_nz); (void)hipFree(g.d_work);
  plk_ntt_free_tables();
  (void)hipStreamDestroy(g.st);
  const int dev = g.device;
  g.~Ctx();
  new (&g) Ctx();
  (void)dev;
}

int plk_dlog_generator(uint8_t out[3]) {
  std::lock_guard<std::mutex> lk(g.mu);
  int rc = ensure();
  if (rc) return rc;
  memcpy(out, g.gen, 3);
  return PLK_OK;
}

int plk_msm_g1(const uint8_t* points, const uint8_t* scalars, size_t n, uint8_t out[3]) {
  if ((!points || !scalars) && n) { plk_set_error("plk_msm_g1: NULL input"); return PLK_ERR_ARG; }
  if (!out) { plk_set_error("plk_msm_g1: NULL out"); return PLK_ERR_ARG; }
  std::lock_guard<std::mutex> lk(g.mu);
  int rc = ensure();
  if (rc) return rc;
  if ((rc = grow(&g.d_pts, &g.cap_pts, 3 * n + 16)) || (rc = grow(&g.d_sc, &g.cap_sc, n + 16))) return rc;
  if (n) {
    PLK_HIP(hipMemcpyAsync(g.d_pts, points, 3 * n, hipMemcpyHostToDevice, g.st));
    PLK_HIP(hipMemcpyAsync(g.d_sc, scalars, n, hipMemcpyHostToDevice, g.st));
  }
  if ((rc = plk_msm_launch(g.d_pts, g.d_sc, n, g.d_res, g.st))) return rc;
  PlkMsmResult h;
  PLK_HIP(hipMemcpyAsync(&h, g.d_res, sizeof h, hipMemcpyDeviceToHost, g.st));
  PLK_HIP(hipStreamSynchronize(g.st));
  if (h.irregular) {
    if ((rc = plk_msm_serial_launch(g.d_pts, g.d_sc, n, g.d_res, g.st))) return rc;
    PLK_HIP(hipMemcpyAsync(&h, g.d_res, sizeof h, hipMemcpyDeviceToHost, g.st));
    PLK_HIP(hipStreamSynchronize(g.st));
  }
  memcpy(out, h.g1, 3);
  return PLK_OK;
}

int plk_poly_mul(const uint8_t* a, size_t la, const uint8_t* b, size_t lb, uint8_t* out, size_t* out_len) {
  if (!out_len) { plk_set_error("plk_poly_mul: NULL out_len"); return PLK_ERR_ARG; }
  if (la == 0 || lb == 0) {
    // reference: calloc(la+lb-1) of zeros, poly_new trims to one zero (or keeps length 0)
    const size_t rl = la + lb - 1;
    if (la + lb == 0) { plk_set_error("plk_poly_mul: both polynomials empty"); return PLK_ERR_ARG; }
    if (rl && out) out[0] = 0;
    *out_len = rl ? 1 : 0;
    return PLK_OK;
  }
  if (!a || !b || !out) { plk_set_error("plk_poly_mul: NULL buffer"); return PLK_ERR_ARG; }
  std::lock_guard<std::mutex> lk(g.mu);
  int rc = ensure();
  if (rc) return rc;
  const size_t rl = la + lb - 1;
  const size_t ws = plk_poly_mul_workspace_bytes(la, lb);
  if ((rc = grow(&g.d_a, &g.cap_a, la + 16)) || (rc = grow(&g.d_b, &g.cap_b, lb + 16)) ||
      (rc = grow(&g.d_out, &g.cap_out, rl + 16)))
    return rc;
  if (ws && (rc = grow((uint8_t**)&g.d_work, &g.cap_work, ws))) return rc;
  PLK_HIP(hipMemcpyAsync(g.d_a, a, la, hipMemcpyHostToDevice, g.st));
  PLK_HIP(hipMemcpyAsync(g.d_b, b, lb, hipMemcpyHostToDevice, g.st));
  if ((rc = plk_poly_mul_launch(g.d_a, la, g.d_b, lb, g.d_out, g.d_nz, g.d_work, g.st))) return rc;
  uint32_t nz = 0;
  PLK_HIP(hipMemcpyAsync(out, g.d_out, rl, hipMemcpyDeviceToHost, g.st));
  PLK_HIP(hipMemcpyAsync(&nz, g.d_nz, 4, hipMemcpyDeviceToHost, g.st));
  PLK_HIP(hipStreamSynchronize(g.st));
  *out_len = nz ? nz : 1;
  return PLK_OK;
}

// ---- device-resident ------------------------------------------------------------------
int plk_msm_result_init(plk_msm_result_t* d_res, void* stream) {
  std::lock_guard<std::mutex> lk(g.mu);
  int rc = ensure();
  if (rc) return rc;
  PLK_HIP(hipMemsetAsync(d_res, 0, sizeof(plk_msm_result_t), pick(stream)));
  return PLK_OK;
}

int plk_msm_g1_dev(const uint8_t* d_points, const uint8_t* d_scalars, size_t n, plk_msm_result_t* d_res,
                   void* stream) {
  int rc = ensure();
  if (rc) return rc;
  return plk_msm_launch(d_points, d_scalars, n, d_res, pick(stream));
}

int plk_msm_g1_batch_dev(const uint8_t* d_points, size_t points_stride, const uint8_t* d_scalars,
                         size_t scalars_stride, size_t n, int batch, plk_msm_result_t* d_res, void* stream) {
  int rc = ensure();
  if (rc) return rc;
  return plk_msm_batch_launch(d_points, points_stride, d_scalars, scalars_stride, n, batch, d_res, pick(stream));
}

int plk_msm_g1_serial_dev(const uint8_t* d_points, const uint8_t* d_scalars, size_t n, plk_msm_result_t* d_res,
                          void* stream) {
  int rc = ensure();
  if (rc) return rc;
  return plk_msm_serial_launch(d_points, d_scalars, n, d_res, pick(stream));
}

int plk_msm_combine_dev(const uint32_t* d_logs, int count, uint8_t* d_out3, void* stream) {
  int rc = ensure();
  if (rc) return rc;
  return plk_msm_combine_launch(d_logs, count, d_out3, pick(stream));
}

int plk_msm_finalize_dev(const uint32_t* d_logs, int batch, int stride, uint8_t* d_out4, void* stream) {
  int rc = ensure();
  if (rc) return rc;
  return plk_msm_finalize_launch(d_logs, batch, stride, d_out4, pick(stream));
}

size_t plk_poly_mul_workspace(size_t la, size_t lb) { return plk_poly_mul_workspace_bytes(la, lb); }

int plk_poly_mul_dev(const uint8_t* d_a, size_t la, const uint8_t* d_b, size_t lb, uint8_t* d_out,
                     uint32_t* d_out_nz, void* d_work, void* stream) {
  int rc = ensure();
  if (rc) return rc;
  return plk_poly_mul_launch(d_a, la, d_b, lb, d_out, d_out_nz, d_work, pick(stream));
}

size_t plk_poly_mul_batch_workspace(const plk_polymul_job_t* jobs, int n) {
  // the size groups run one after another on the stream and reuse the workspace: the largest
  // group's need (jobs of one size 2^k take 2^(k+3) bytes each)
  size_t per_k[64] = {0}, best = 0;
  for (int i = 0; jobs && i < n; i++) {
    const size_t w = plk_poly_mul_workspace_bytes(jobs[i].la, jobs[i].lb);
    if (!w) continue;
    int k = 0;
    while (((size_t)8 << k) < w) k++;
    per_k[k] += w;
    best = per_k[k] > best ? per_k[k] : best;
  }
  return best;
}

int plk_poly_mul_batch_dev(const plk_polymul_job_t* jobs, int n, void* d_work, size_t work_bytes, void* stream) {
  int rc = ensure();
  if (rc) return rc;
  if (!jobs || n < 1 || n > 64) {
    plk_set_error("plk_poly_mul_batch_dev: %d jobs (1..64)", n);
    return PLK_ERR_ARG;
  }
  PlkPolyMulJob js[64];
  for (int i = 0; i < n; i++) {
    if (!jobs[i].a || !jobs[i].b || !jobs[i].out) {
      plk_set_error("plk_poly_mul_batch_dev: null buffer in job %d", i);
      return PLK_ERR_ARG;
    }
    js[i] = PlkPolyMulJob{jobs[i].a, jobs[i].la, jobs[i].b, jobs[i].lb, jobs[i].out, jobs[i].acc ? 1 : 0};
  }
  return plk_poly_mul_batch_launch(js, n, d_work, work_bytes, pick(stream));
}

int plk_ntt_dev(uint32_t* d_data, int log_n, int inverse, void* stream) {
  int rc = ensure();
  if (rc) return rc;
  return plk_ntt_launch(d_data, log_n, 1, inverse, pick(stream));
}

int plk_ntt_batch_dev(uint32_t* d_data, int log_n, int batch, int inverse, void* stream) {
  int rc = ensure();
  if (rc) return rc;
  if (!d_data || batch < 1) {
    plk_set_error("plk_ntt_batch_dev: null data or batch %d", batch);
    return PLK_ERR_ARG;
  }
  return plk_ntt_launch(d_data, log_n, batch, inverse, pick(stream));
}

}  // extern "C"
